"""``newton_krylov`` drop-in: SciPy's call surface, libnkhip's device solver underneath.

Mirrors ``scipy.optimize.newton_krylov`` (scipy/optimize/_nonlin.py:1553-1603; called by the
reference at sh_scipy_nk.py:61, sh_vscode_nk.py:59, PMA2_nk.py:100, droplet.py:383):

* same keyword arguments and defaults (f_tol = eps^(1/3) on the max-norm, inner_m = 30,
  outer_k = 10, Armijo line search, Eisenstat-Walker forcing);
* ``xin`` is not modified, a new array shaped like ``xin`` is returned;
* ``NoConvergence`` (carrying the last iterate) when ``maxiter`` is hit, ``ValueError`` for a
  zero Newton step or a non-finite Jacobian-vector product;
* ``verbose`` prints ``"%d:  |F(x)| = %g; step %g"`` per Newton iteration.

``F`` receives and returns float64 torch tensors on the GPU (shaped like ``xin``); it is called
synchronously from the solver, re-entrantly from the JVP and the line search, exactly like the
reference's closures.  Every vector the Krylov method touches stays in HBM.
"""
from __future__ import annotations

import ctypes as C
import math

import numpy as np
import torch

from . import _lib
from ._lib import check, lib

try:  # let `except scipy.optimize.NoConvergence` keep working for drop-in users
    from scipy.optimize import NoConvergence as _ScipyNoConvergence
except Exception:  # pragma: no cover - scipy is optional for the product
    _ScipyNoConvergence = Exception


class NoConvergence(_ScipyNoConvergence):
    """Raised when the nonlinear solver hits ``maxiter`` (scipy/optimize/_nonlin.py:30-33)."""


def make_opts(*, rdiff=None, inner_maxiter=20, outer_k=10, verbose=False, maxiter=None,
              f_tol=None, f_rtol=None, x_tol=None, x_rtol=None, line_search="armijo",
              inner_m=30, jvp="fd", profile=False) -> _lib.nk_opts:
    o = _lib.default_opts()
    nan = float("nan")
    o.f_tol = nan if f_tol is None else float(f_tol)
    o.f_rtol = nan if f_rtol is None else float(f_rtol)
    o.x_tol = nan if x_tol is None else float(x_tol)
    o.x_rtol = nan if x_rtol is None else float(x_rtol)
    o.rdiff = 0.0 if rdiff is None else float(rdiff)
    o.maxiter = 0 if maxiter is None else int(maxiter)
    o.inner_m = int(inner_m)
    o.outer_k = int(outer_k)
    if line_search is True:
        line_search = "armijo"
    if line_search in (False, None):
        o.line_search = 0
    elif line_search == "armijo":
        o.line_search = 1
    else:
        raise NotImplementedError(f"line_search={line_search!r}: only 'armijo' and None are built")
    if jvp not in ("fd", "analytic"):
        raise ValueError("jvp must be 'fd' (scipy-faithful) or 'analytic'")
    o.jvp_mode = _lib.NK_JVP_FD if jvp == "fd" else _lib.NK_JVP_ANALYTIC
    o.verbose = 1 if verbose else 0
    # profile: False/0 off, True/1 every launch timed, k > 1 every k-th launch of each class
    o.profile = int(profile) if not isinstance(profile, bool) else (1 if profile else 0)
    # inner_maxiter is the LGMRES outer-cycle count, which KrylovJacobian overrides to 1
    # (_nonlin.py:1483), so it has no effect -- accepted for signature compatibility.
    del inner_maxiter
    return o


def raise_for_status(rc: int, x_last=None):
    if rc == _lib.NK_OK:
        return
    if rc == _lib.NK_NO_CONVERGENCE:
        raise NoConvergence(x_last)
    if rc == _lib.NK_NONFINITE:
        raise ValueError("Function returned non-finite results")
    if rc == _lib.NK_BAD_RHS:
        raise ValueError("RHS must contain only finite numbers")
    if rc == _lib.NK_ZERO_STEP:
        raise ValueError("Jacobian inversion yielded zero vector. "
                         "This indicates a bug in the Jacobian approximation.")
    check(rc, "libnkhip")


class _Views:
    """Maps the device pointers libnkhip hands to F back onto torch views."""

    def __init__(self, shape, n, tensors):
        self.shape = shape
        self.n = n
        self.spans = [(t.data_ptr(), t.data_ptr() + t.numel() * 8, t) for t in tensors]

    def view(self, ptr):
        for lo, hi, t in self.spans:
            if lo <= ptr < hi:
                off = (ptr - lo) // 8
                return t.view(-1)[off:off + self.n].view(self.shape)
        raise RuntimeError("libnkhip passed a pointer outside the known buffers")


def newton_krylov(F, xin, iter=None, rdiff=None, method="lgmres", inner_maxiter=20,
                  inner_M=None, outer_k=10, verbose=False, maxiter=None, f_tol=None, f_rtol=None,
                  x_tol=None, x_rtol=None, tol_norm=None, line_search="armijo", callback=None,
                  *, full_output=False, **kw):
    """Find a root of ``F`` with inexact Newton-Krylov on the GPU (scipy signature)."""
    if method != "lgmres":
        raise NotImplementedError("only method='lgmres' (the scipy default) is built")
    if inner_M is not None or tol_norm is not None or iter is not None or callback is not None:
        raise NotImplementedError("inner_M / tol_norm / iter / callback are not supported")
    inner_m = kw.pop("inner_inner_m", 30)
    if kw:
        raise ValueError(f"Unknown parameter {next(iter_keys(kw))}")
    o = make_opts(rdiff=rdiff, outer_k=outer_k, verbose=verbose, maxiter=maxiter, f_tol=f_tol,
                  f_rtol=f_rtol, x_tol=x_tol, x_rtol=x_rtol, line_search=line_search,
                  inner_m=inner_m)

    as_numpy = not isinstance(xin, torch.Tensor)
    x0 = (torch.as_tensor(np.asarray(xin, dtype=np.float64)) if as_numpy else xin)
    x0 = x0.to(device="cuda", dtype=torch.float64).contiguous().clone()
    shape = x0.shape
    n = x0.numel()
    x = torch.empty_like(x0)
    ws_bytes = check(int(lib.nk_solve_workspace_bytes(n, C.byref(o))), "workspace size")
    ws = torch.empty(ws_bytes // 8 + 64, dtype=torch.float64, device="cuda")
    base = ws.data_ptr()
    shift = (-base) % 256 // 8
    ws_al = ws[shift:]
    views = _Views(shape, n, [x0, x, ws_al])
    err = []

    def _cb(_ctx, xp, fp, nn):
        try:
            xv = views.view(xp)
            fv = views.view(fp)
            r = F(xv)
            r = torch.as_tensor(r, device="cuda", dtype=torch.float64)
            fv.copy_(r.reshape(shape))
            return 0
        except BaseException as e:  # noqa: BLE001 - re-raised after the C call returns
            err.append(e)
            return 1

    cfn = _lib.RESIDUAL_FN(_cb)
    st = _lib.nk_stats()
    stream = C.c_void_p(torch.cuda.current_stream().cuda_stream)
    rc = lib.nk_solve(cfn, None, C.c_void_p(x0.data_ptr()), C.c_void_p(x.data_ptr()), n,
                      C.byref(o), C.byref(st), stream, C.c_void_p(ws_al.data_ptr()),
                      ws_al.numel() * 8)
    if err:
        raise err[0]
    out = x.cpu().numpy().reshape(np.shape(xin)) if as_numpy else x.reshape(shape)
    if rc == _lib.NK_NO_CONVERGENCE:
        raise NoConvergence(out)
    raise_for_status(rc)
    if full_output:
        return out, st.as_dict()
    return out


def iter_keys(d):
    return iter(d.keys())
