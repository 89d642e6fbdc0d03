"""MEMS deflection on a moving mesh: python_work/PMA2_nk.py's time-stepper over libnkhip.

The reference keeps its state in module globals (``U.new``, ``Q.val``) and advances it in the
``while current_time < Tf`` loop of ``main()`` (:77-106):

    U.val = U.new; mesh fields; J; compute_u_spatial_ders
    dt = compute_g()*k                        # min((1+u)^3) k: moves the mesh and the clock
    solve_PMA(); CN_term = compute_rhs_pde()
    U.new = newton_krylov(residual, U.val, verbose=0)    # residual() divides by the GLOBAL dt = k
    Q.val += dt*Q.dt

``Mems.step`` is that loop body on the GPU: single-workgroup HIP kernels for the bilaplacian
residual (two Laplace_operator applications per evaluation), the shared Newton-Krylov core, and
one monitor / DCT mesh step.  Only p = 2 exists: the reference's p = 1 branch raises (:135).
"""
from __future__ import annotations

import ctypes as C

import numpy as np
import torch

from . import _lib
from ._lib import check, lib
from .droplet import FIELDS as _DROP_FIELDS
from .solver import NoConvergence, make_opts, raise_for_status

FIELDS = dict(_DROP_FIELDS)
FIELDS.pop("F")
FIELDS["CN"] = 9


class Mems:
    """The PMA2_nk.py stepper; keyword arguments override the module globals (:22-37):
    n (N_), p (p_), m (m_), alpha (alpha_), gamma (gamma_), epsilon (epsilon_), beta (beta_),
    smoothing_iters, lambd (lambd_), endl, endr, k."""

    def __init__(self, *, maxiter=None, f_tol=None, verbose=False, profile=False, stream=None,
                 **params):
        p = _lib.nk_mems_params()
        lib.nk_mems_params_default(C.byref(p))
        for key, v in params.items():
            if not hasattr(p, key):
                raise ValueError(f"unknown PMA2 parameter {key}")
            setattr(p, key, v)
        if p.p != 2:
            raise ValueError("only p = 2 is defined: the reference's p = 1 residual raises "
                             "(PMA2_nk.py:135)")
        self.params = p
        self.n = p.n
        self.nn = p.n * p.n
        self.opts = make_opts(maxiter=maxiter, f_tol=f_tol, verbose=verbose, profile=profile)
        self._stream = stream
        self._h = C.c_void_p()
        check(lib.nk_mems_create(C.byref(self._h), C.byref(p), C.byref(self.opts), self._sp()),
              "nk_mems_create")
        self.time = 0.0
        self.last_stats = None
        self.set_state(*self.initial_state())

    def _sp(self):
        st = self._stream if self._stream is not None else torch.cuda.current_stream()
        return C.c_void_p(st.cuda_stream)

    def close(self):
        if self._h:
            lib.nk_mems_destroy(self._h)
            self._h = C.c_void_p()

    def __del__(self):  # pragma: no cover
        try:
            self.close()
        except Exception:
            pass

    def _dev(self, a):
        t = a if isinstance(a, torch.Tensor) else torch.as_tensor(np.asarray(a, dtype=np.float64))
        t = t.to(device="cuda", dtype=torch.float64).contiguous().reshape(-1)
        if t.numel() != self.nn:
            raise ValueError(f"expected {self.nn} values, got {t.numel()}")
        return t

    # ------------------------------------------------------------------ state
    def initial_state(self):
        """main() initialisation (:65-71): Q = (xi^2 + eta^2)/2 on the grid, U = 0."""
        ksi = np.linspace(self.params.endl, self.params.endr, self.n)
        kk, ee = np.meshgrid(ksi, ksi)
        return np.zeros(self.nn), np.reshape(0.5 * kk ** 2 + 0.5 * ee ** 2, self.nn)

    def set_state(self, U, Q):
        u, q = self._dev(U), self._dev(Q)
        check(lib.nk_mems_set_state(self._h, C.c_void_p(u.data_ptr()), C.c_void_p(q.data_ptr())),
              "nk_mems_set_state")
        self.time = 0.0

    def state(self):
        u = torch.empty(self.nn, dtype=torch.float64, device="cuda")
        q = torch.empty_like(u)
        check(lib.nk_mems_get_state(self._h, C.c_void_p(u.data_ptr()), C.c_void_p(q.data_ptr())),
              "nk_mems_get_state")
        return u, q

    # ------------------------------------------------------------------ stepping
    def step(self):
        """One pass of main()'s loop (:77-103); returns the adaptive dt."""
        st = _lib.nk_stats()
        dt, tm = C.c_double(), C.c_double()
        rc = lib.nk_mems_step(self._h, C.byref(st), C.byref(dt), C.byref(tm))
        self.last_stats = st.as_dict()
        if rc == _lib.NK_NO_CONVERGENCE:
            raise NoConvergence(self.state()[0])
        raise_for_status(rc)
        self.time = tm.value
        return dt.value

    def run(self, Tf=0.3, max_steps=None):
        """``while current_time < Tf`` (:77); returns the list of dt."""
        dts = []
        while self.time < Tf and (max_steps is None or len(dts) < max_steps):
            dts.append(self.step())
        return dts

    # ------------------------------------------------------------------ pieces (tests)
    def prepare(self):
        """:80-94 for the current state (U.val = U.new); returns compute_g()*k."""
        dt = C.c_double()
        check(lib.nk_mems_prepare(self._h, C.byref(dt)), "nk_mems_prepare")
        return dt.value

    def field(self, name):
        out = torch.empty(self.nn, dtype=torch.float64, device="cuda")
        check(lib.nk_mems_field(self._h, FIELDS[name], C.c_void_p(out.data_ptr())),
              "nk_mems_field")
        return out

    def residual(self, u):
        u = self._dev(u)
        out = torch.empty_like(u)
        check(lib.nk_mems_residual(self._h, C.c_void_p(u.data_ptr()), C.c_void_p(out.data_ptr())),
              "nk_mems_residual")
        return out
