"""Thin-film droplet coalescence on a moving mesh: python_work/droplet.py's stepper over libnkhip.

The reference (``droplet.py``) keeps its state in module globals (``U.val``/``U.new``, ``Q.val``)
and advances it with ``evolve_with_PDE(dt, iterMax, tol, dtmesh, pmaloops)`` (:360-411):

    dt_n = dt*scale; U.val = U.new
    mesh / old-time fields (:372-381)
    U.new = newton_krylov(lambda u: residual(u, F, dt_n), U.val, verbose=1, maxiter=20, f_tol=1e-7)
    loop_pma(dtmesh, pmaloops)                         # moving mesh, 80 % of the CPU time
    scale += exp(-10*|U.new - U.val|)

``Droplet.step`` is that loop body on the GPU: one single-workgroup kernel per residual
evaluation, the shared Newton-Krylov core, and the whole PMA mesh loop in one persistent kernel.
``read_init`` / ``write_init`` handle the reference's ``initdrop_*.txt`` state files.
"""
from __future__ import annotations

import ctypes as C
import math
import os

import numpy as np
import torch

from . import _lib
from ._lib import check, lib
from .solver import NoConvergence, make_opts, raise_for_status

FIELDS = {"d2ksi": 0, "d2eta": 1, "dksideta": 2, "J": 3, "A11": 4, "A22": 5, "A12": 6,
          "Q_dksi": 7, "Q_deta": 8, "F": 9, "U_xx": 10, "U_yy": 11, "U_val": 12, "U_new": 13,
          "Q_val": 14}


def init_filename(R=1, Nx=91, Ny=61, a=100, epsilon=0.01, alpha=0.01, gamma=0.1, C_=0.15,
                  kind="coal"):
    """The reference's naming convention (droplet.py:137-138, :186-188)."""
    return f"initdrop_{kind}_{R}_{Nx}-{Ny}_{a}_{epsilon}_{alpha}_{gamma}_{C_}.txt"


def read_init(path):
    """read_from_file (:564-576): one 'U Q' pair per line, NN lines, row-major (eta rows)."""
    d = np.loadtxt(path)
    return d[:, 0].copy(), d[:, 1].copy()


def write_init(path, U, Q):
    """write_to_file (:556-562): str(U[i]) + ' ' + str(Q[i]) per line."""
    U = np.asarray(U, dtype=np.float64).reshape(-1)
    Q = np.asarray(Q, dtype=np.float64).reshape(-1)
    with open(path, "w") as fh:
        for u, q in zip(U, Q):
            fh.write(str(u) + " " + str(q) + "\n")


class Droplet:
    """The droplet.py stepper; keyword arguments override the module globals (:22-53)."""

    def __init__(self, *, maxiter=20, f_tol=1e-7, verbose=False, profile=False, stream=None,
                 **params):
        p = _lib.nk_drop_params()
        lib.nk_drop_params_default(C.byref(p))
        for k, v in params.items():
            if not hasattr(p, k):
                raise ValueError(f"unknown droplet parameter {k}")
            setattr(p, k, v)
        self.params = p
        self.nx, self.ny = p.nx, p.ny
        self.n = p.nx * p.ny
        self.opts = make_opts(maxiter=maxiter, f_tol=f_tol, verbose=verbose, profile=profile)
        self._stream = stream
        self._h = C.c_void_p()
        check(lib.nk_drop_create(C.byref(self._h), C.byref(p), C.byref(self.opts),
                                 self._sp()), "nk_drop_create")
        self.scale = 1.0
        self.time = 0.0
        self.last_stats = None

    def _sp(self):
        st = self._stream if self._stream is not None else torch.cuda.current_stream()
        return C.c_void_p(st.cuda_stream)

    def close(self):
        if self._h:
            lib.nk_drop_destroy(self._h)
            self._h = C.c_void_p()

    def __del__(self):  # pragma: no cover
        try:
            self.close()
        except Exception:
            pass

    def _dev(self, a):
        t = torch.as_tensor(np.asarray(a, dtype=np.float64) if not isinstance(a, torch.Tensor) else a)
        t = t.to(device="cuda", dtype=torch.float64).contiguous().reshape(-1)
        if t.numel() != self.n:
            raise ValueError(f"expected {self.n} values, got {t.numel()}")
        return t

    # ------------------------------------------------------------------ state
    def set_state(self, U, Q, scale=1.0):
        u, q = self._dev(U), self._dev(Q)
        check(lib.nk_drop_set_state(self._h, C.c_void_p(u.data_ptr()), C.c_void_p(q.data_ptr())),
              "nk_drop_set_state")
        self.scale = float(scale)
        check(lib.nk_drop_set_scale(self._h, self.scale), "nk_drop_set_scale")

    def state(self):
        u = torch.empty(self.n, dtype=torch.float64, device="cuda")
        q = torch.empty_like(u)
        check(lib.nk_drop_get_state(self._h, C.c_void_p(u.data_ptr()), C.c_void_p(q.data_ptr())),
              "nk_drop_get_state")
        return u, q

    def load_init(self, path):
        self.set_state(*read_init(path))

    def initial_state(self):
        """main() (:103-106): U = epsilon everywhere, Q = (xi^2 + eta^2)/2 on the grid."""
        p = self.params
        kk, ee = np.meshgrid(np.linspace(p.endl, p.endr, p.nx), np.linspace(p.endb, p.endt, p.ny))
        return np.full(self.n, p.epsilon), np.reshape(0.5 * kk ** 2 + 0.5 * ee ** 2, self.n)

    def initialise_coalescing(self, vsteps=1000, info=((0, 0, 1, 1), (3, 0, 1, 1)),
                              dtmesh=5e-9, loops=20, tofile=None):
        """initialise_coalescing_droplets(Vsteps, info, dtmesh, loops, False, tofile)
        (droplet.py:132-189) from main()'s initial state: the droplets' volumes grow linearly
        over `vsteps` steps, each followed by loop_pma(dtmesh, loops).  `tofile`: a directory to
        write the reference's initdrop_coal_*.txt into (None: no file)."""
        self.set_state(*self.initial_state())
        rows = np.ascontiguousarray(np.asarray(info, dtype=np.float64).reshape(-1, 4))
        check(lib.nk_drop_init_coalescing(
            self._h, int(vsteps), rows.ctypes.data_as(C.POINTER(C.c_double)), rows.shape[0],
            float(dtmesh), int(loops)), "nk_drop_init_coalescing")
        U, Q = self.state()
        if tofile is not None:
            p = self.params
            name = init_filename(R=1, Nx=p.nx, Ny=p.ny, a=int(p.a) if float(p.a).is_integer()
                                 else p.a, epsilon=p.epsilon, alpha=p.alpha, gamma=p.gamma,
                                 C_=p.C)
            write_init(os.path.join(tofile, name), U.cpu().numpy(), Q.cpu().numpy())
        return U, Q

    # ------------------------------------------------------------------ stepping
    def step(self, dt=1e-4, dtmesh=3e-9, pmaloops=400):
        """One iteration of evolve_with_PDE's loop (droplet.py:369-411)."""
        st = _lib.nk_stats()
        dtu, sc = C.c_double(), C.c_double()
        rc = lib.nk_drop_step(self._h, float(dt), float(dtmesh), int(pmaloops), C.byref(st),
                              C.byref(dtu), C.byref(sc))
        self.last_stats = st.as_dict()
        if rc == _lib.NK_NO_CONVERGENCE:
            raise NoConvergence(self.state()[0])
        raise_for_status(rc)
        self.scale = sc.value
        self.time += dtu.value
        return dtu.value

    def evolve(self, nsteps, dt=1e-4, dtmesh=3e-9, pmaloops=400):
        return [self.step(dt, dtmesh, pmaloops) for _ in range(int(nsteps))]

    # ------------------------------------------------------------------ pieces (tests)
    def prepare(self):
        check(lib.nk_drop_prepare(self._h), "nk_drop_prepare")

    def field(self, name):
        out = torch.empty(self.n, dtype=torch.float64, device="cuda")
        check(lib.nk_drop_field(self._h, FIELDS[name], C.c_void_p(out.data_ptr())), "nk_drop_field")
        return out

    def residual(self, u, dt):
        u = self._dev(u)
        out = torch.empty_like(u)
        check(lib.nk_drop_residual(self._h, C.c_void_p(u.data_ptr()), float(dt),
                                   C.c_void_p(out.data_ptr())), "nk_drop_residual")
        return out

    def solve(self, dt):
        out = torch.empty(self.n, dtype=torch.float64, device="cuda")
        st = _lib.nk_stats()
        rc = lib.nk_drop_solve(self._h, float(dt), C.c_void_p(out.data_ptr()), C.byref(st))
        self.last_stats = st.as_dict()
        if rc == _lib.NK_NO_CONVERGENCE:
            raise NoConvergence(out)
        raise_for_status(rc)
        return out

    def pma(self, dtmesh, loops):
        check(lib.nk_drop_pma(self._h, float(dtmesh), int(loops)), "nk_drop_pma")
