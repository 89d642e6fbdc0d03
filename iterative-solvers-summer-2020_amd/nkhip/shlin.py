"""Semi-implicit Swift-Hohenberg stepper: python_work/sh_linearised.py over libnkhip.

The reference's ``main()`` (:14-65) advances U with one sparse direct solve per step,

    D = diags((5U - Uo)^2 k/16 - g k U);  Uo = U
    U = spsolve(I + D - L k/2, (I + L k/2) Uo)                                      (:48-56)

starting from ``Uo = U`` (:25-26).  ``SHLinearised.step`` performs the same step on the GPU with a
matrix-free conjugate-gradient solve over the 13-point stencil kernel (the system is symmetric
positive definite for g = 0, the reference's value), warm-started from U and run to a relative
residual of ``rtol``.
"""
from __future__ import annotations

import ctypes as C

import torch

from ._lib import NK_NO_CONVERGENCE, check, lib
from .solver import NoConvergence, raise_for_status


class SHLinearised:
    def __init__(self, N=64, d=40.0, k=0.2, r=0.2, g=0.0, *, ny=None, rtol=1e-14, maxiter=1000,
                 stream=None):
        self.N = int(N)
        self.ny = int(ny) if ny is not None else self.N
        self.h = float(d) / self.N  # h = d/N (:18)
        self.k, self.r, self.g = float(k), float(r), float(g)
        self._stream = stream
        self._h = C.c_void_p()
        st = stream if stream is not None else torch.cuda.current_stream()
        check(lib.nk_shlin_create(C.byref(self._h), self.ny, self.N, self.h, self.r, self.g,
                                  self.k, float(rtol), int(maxiter), C.c_void_p(st.cuda_stream)),
              "nk_shlin_create")
        self.last_iters = 0
        self.last_relres = 0.0

    def close(self):
        if self._h:
            lib.nk_shlin_destroy(self._h)
            self._h = C.c_void_p()

    def __del__(self):  # pragma: no cover
        try:
            self.close()
        except Exception:
            pass

    def _dev(self, a):
        t = torch.as_tensor(a).to(device="cuda", dtype=torch.float64).contiguous().reshape(-1)
        if t.numel() != self.ny * self.N:
            raise ValueError(f"expected {self.ny * self.N} values, got {t.numel()}")
        return t

    def step(self, U, Uo):
        """U[s+1] from U = U[s], Uo = U[s-1] (:48-56)."""
        U, Uo = self._dev(U), self._dev(Uo)
        out = torch.empty_like(U)
        its, rel = C.c_int64(), C.c_double()
        rc = lib.nk_shlin_step(self._h, C.c_void_p(U.data_ptr()), C.c_void_p(Uo.data_ptr()),
                               C.c_void_p(out.data_ptr()), C.byref(its), C.byref(rel))
        self.last_iters, self.last_relres = its.value, rel.value
        if rc == NK_NO_CONVERGENCE:
            raise NoConvergence(out)
        raise_for_status(rc)
        return out

    def run(self, U0, nsteps):
        """main()'s loop from Uo = U = U0 (:25-26, :46-56); returns [U[1], ..., U[nsteps]]."""
        U = self._dev(U0)
        Uo, out = U, []
        for _ in range(int(nsteps)):
            U, Uo = self.step(U, Uo), U
            out.append(U)
        return out
