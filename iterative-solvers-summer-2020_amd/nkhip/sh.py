"""Swift-Hohenberg Crank-Nicolson stepper: the reference's call surface over libnkhip.

The reference script ``python_work/sh_scipy_nk.py`` (and its duplicate ``sh_vscode_nk.py``, and
the C++ twin ``cpp_work/.../main.cpp``) is a module-level loop:

    L = -Lap*Lap - 2*Lap + (r-1)*I                       # :38-39
    for s in range(Nsteps):                              # :53
        Uo = U.copy(); UoUo = Uo*Uo; UoUoUo = Uo*UoUo    # :56-58
        U = newton_krylov(residual, Uo, verbose=1)       # :61

``SwiftHohenberg`` keeps those parameters (d, N, h = d/N, k, r, g; defaults = the reference
constants :15-29) and ``step(U)`` is the loop body: hand in a 2-D grid state, get the next
implicit time step.  The whole Newton-Krylov solve runs on the GPU (nk_sh_step): the residual,
the finite-difference JVP and the Arnoldi BLAS-1 work are HIP kernels, the host keeps scalars.
"""
from __future__ import annotations

import ctypes as C
import math

import torch

from . import _lib
from ._lib import check, lib
from .solver import make_opts, raise_for_status, NoConvergence  # noqa: F401


class SwiftHohenberg:
    """u_t = r u - (1 + lap)^2 u + g u^2 - u^3 on a periodic N x N torus (sh_scipy_nk.py)."""

    def __init__(self, N: int = 64, d: float = 40.0, k: float = 0.2, r: float = 0.01,
                 g: float = 1.0, *, ny: int | None = None, jvp: str = "fd", f_tol=None,
                 f_rtol=None, x_tol=None, x_rtol=None, maxiter=None, rdiff=None, outer_k=10,
                 inner_m=30, line_search="armijo", verbose=False, profile=False,
                 comm=None, ny_local: int | None = None, stream=None):
        self.N = int(N)          # points in x (and in y unless ny is given)
        self.nx = int(N)
        self.ny = int(ny) if ny is not None else int(N)
        self.d = float(d)
        self.h = self.d / self.N  # sh_scipy_nk.py:17
        self.k = float(k)
        self.r = float(r)
        self.g = float(g)
        self.e = 1.0 / self.h ** 2  # :32
        self.comm = comm
        self.ny_local = int(ny_local) if ny_local is not None else self.ny
        self.opts = make_opts(rdiff=rdiff, outer_k=outer_k, verbose=verbose, maxiter=maxiter,
                              f_tol=f_tol, f_rtol=f_rtol, x_tol=x_tol, x_rtol=x_rtol,
                              line_search=line_search, inner_m=inner_m, jvp=jvp,
                              profile=profile)
        self._stream = stream
        self._h = C.c_void_p()
        s = self._stream_ptr()
        check(lib.nk_sh_create(C.byref(self._h), self.ny_local, self.nx, self.ny, self.h, self.r,
                               self.k, self.g, C.byref(self.opts),
                               comm.handle if comm is not None else None, s), "nk_sh_create")
        self.last_stats = None

    def _stream_ptr(self):
        st = self._stream if self._stream is not None else torch.cuda.current_stream()
        return C.c_void_p(st.cuda_stream)

    def close(self):
        if self._h:
            lib.nk_sh_destroy(self._h)
            self._h = C.c_void_p()

    def __del__(self):  # pragma: no cover - interpreter shutdown order
        try:
            self.close()
        except Exception:
            pass

    # ----------------------------------------------------------------------------- options
    def set_options(self, **kw):
        o = make_opts(**kw)
        check(lib.nk_sh_set_opts(self._h, C.byref(o)), "nk_sh_set_opts")
        self.opts = o

    # ----------------------------------------------------------------------------- stepping
    def _as_grid(self, U):
        U = torch.as_tensor(U)
        if U.device.type != "cuda" or U.dtype != torch.float64:
            U = U.to(device="cuda", dtype=torch.float64)
        return U.contiguous()

    def step(self, U, out=None):
        """One implicit Crank-Nicolson step U[s] -> U[s+1] (sh_scipy_nk.py:56-61).

        ``out`` (optional) must be a contiguous float64 CUDA tensor with as many values as the
        slab; it may alias ``U``.  The library runs on the stepper's stream: when that is not
        torch's current stream, it first waits for the work torch has queued (U, out), and torch's
        stream waits for the step before anything reads ``out``."""
        U = self._as_grid(U)
        if U.numel() != self.ny_local * self.nx:
            raise ValueError(f"state has {U.numel()} values, slab is {self.ny_local}x{self.nx}")
        if out is None:
            out = torch.empty_like(U)
        elif (not isinstance(out, torch.Tensor) or out.device.type != "cuda"
              or out.device != U.device or out.dtype != torch.float64
              or out.numel() != U.numel() or not out.is_contiguous()):
            raise ValueError("out must be a contiguous float64 CUDA tensor on the state's device "
                             f"with {U.numel()} values")
        cur = torch.cuda.current_stream(U.device)
        mine = self._stream if self._stream is not None else cur
        if mine != cur:
            mine.wait_stream(cur)
        st = _lib.nk_stats()
        rc = lib.nk_sh_step(self._h, C.c_void_p(U.data_ptr()), C.c_void_p(out.data_ptr()),
                            C.byref(st))
        if mine != cur:
            cur.wait_stream(mine)
        self.last_stats = st.as_dict()
        if rc == _lib.NK_NO_CONVERGENCE:
            raise NoConvergence(out)
        raise_for_status(rc)
        return out

    def run(self, U, nsteps: int):
        """``nsteps`` implicit steps (the loop of sh_scipy_nk.py:53-61 without plotting)."""
        U = self._as_grid(U)
        a, b = U.clone(), torch.empty_like(U)
        for _ in range(int(nsteps)):
            self.step(a, out=b)
            a, b = b, a
        return a

    # ----------------------------------------------------------------------------- operators
    def L(self, v):
        from .ops import sh13_apply
        return sh13_apply(self._as_grid(v), self.h, self.r, self.ny, self.nx)

    def Lap(self, v):
        from .ops import lap5_apply
        return lap5_apply(self._as_grid(v), self.e, self.ny, self.nx)

    def residual(self, u, Uo):
        """``residual(u)`` with the module global ``Uo`` made explicit (sh_scipy_nk.py:47-49)."""
        from .ops import sh_residual
        return sh_residual(self._as_grid(u), self._as_grid(Uo), self.h, self.r, self.k, self.g,
                           self.ny, self.nx)

    # ----------------------------------------------------------------------------- profiling
    def kernel_profile(self):
        recs = (_lib.nk_kprof * 32)()
        n = check(lib.nk_sh_kernel_profile(self._h, recs, 32), "nk_sh_kernel_profile")
        return {recs[i].name.decode(): {"launches": recs[i].launches, "ms": recs[i].total_ms,
                                        "alg_bytes": recs[i].alg_bytes, "timed": recs[i].timed,
                                        "timed_bytes": recs[i].timed_bytes} for i in range(n)}

    def reset_profile(self):
        check(lib.nk_sh_reset_profile(self._h), "nk_sh_reset_profile")

    def workspace_bytes(self) -> int:
        return int(lib.nk_sh_workspace_bytes(self._h))

    def step_log(self):
        """The accepted Armijo step of every Newton iteration of the last step (the ``step %g``
        column of the reference's verbose output, sh_scipy_nk.py:61)."""
        n = check(lib.nk_sh_step_log(self._h, None, 0), "nk_sh_step_log")
        buf = (C.c_double * max(n, 1))()
        check(lib.nk_sh_step_log(self._h, buf, n), "nk_sh_step_log")
        return [buf[i] for i in range(n)]


def sh_step(U, h, k=0.2, r=0.01, g=1.0, **kw):
    """Functional form: the next implicit step of a 2-D periodic grid with mesh spacing h."""
    U = torch.as_tensor(U)
    ny, nx = U.shape
    model = SwiftHohenberg(N=nx, d=h * nx, k=k, r=r, g=g, ny=ny, **kw)
    try:
        return model.step(U)
    finally:
        model.close()
