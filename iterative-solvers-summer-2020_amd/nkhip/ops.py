"""Device operators over PyTorch-ROCm fp64 tensors, each one call into libnkhip.

These replace the pieces of ``python_work/sh_scipy_nk.py`` one by one:
``lap5_apply`` = ``Lap @ v`` (:32-35), ``sh13_apply`` = ``L @ v`` (:38-39), ``sh_residual`` =
``residual(u)`` (:47-49), and the BLAS-1 calls SciPy's Arnoldi makes
(scipy/sparse/linalg/_isolve/_gcrotmk.py:104-143).  Tensors must be CUDA (HIP) float64; the
kernels run on torch's current stream.
"""
from __future__ import annotations

import ctypes as C

import torch

from ._lib import check, lib


def _stream():
    return C.c_void_p(torch.cuda.current_stream().cuda_stream)


def _dev(t: torch.Tensor, name: str) -> torch.Tensor:
    if not isinstance(t, torch.Tensor) or not t.is_cuda:
        raise TypeError(f"{name} must be a CUDA (HIP) tensor")
    if t.dtype != torch.float64:
        raise TypeError(f"{name} must be float64 (the reference computes in fp64)")
    if not t.is_contiguous():
        raise ValueError(f"{name} must be contiguous")
    return t


def _ptr(t: torch.Tensor):
    return C.c_void_p(t.data_ptr())


def _grid(v: torch.Tensor, ny, nx):
    if ny is None or nx is None:
        if v.dim() != 2:
            raise ValueError("pass a 2-D (ny, nx) grid or ny/nx explicitly")
        ny, nx = v.shape
    if v.numel() != ny * nx:
        raise ValueError(f"grid {ny}x{nx} does not match {v.numel()} values")
    return int(ny), int(nx)


def lap5_apply(v, e, ny=None, nx=None, out=None):
    """``Lap @ v``: periodic 5-point Laplacian with e = 1/h^2 (sh_scipy_nk.py:32-35)."""
    _dev(v, "v")
    ny, nx = _grid(v, ny, nx)
    out = torch.empty_like(v) if out is None else _dev(out, "out")
    check(lib.nk_lap5_apply(_ptr(v), _ptr(out), ny, nx, float(e), _stream()), "nk_lap5_apply")
    return out


def sh13_apply(v, h, r, ny=None, nx=None, out=None):
    """``L @ v`` with L = -Lap*Lap - 2*Lap + (r-1)*I (sh_scipy_nk.py:38-39)."""
    _dev(v, "v")
    ny, nx = _grid(v, ny, nx)
    out = torch.empty_like(v) if out is None else _dev(out, "out")
    check(lib.nk_sh13_apply(_ptr(v), _ptr(out), ny, nx, float(h), float(r), _stream()),
          "nk_sh13_apply")
    return out


def sh_residual(u, uo, h, r, k, g, ny=None, nx=None, out=None):
    """``residual(u)`` of sh_scipy_nk.py:47-49 with ``Uo = uo``, fused into one pass."""
    _dev(u, "u")
    _dev(uo, "uo")
    ny, nx = _grid(u, ny, nx)
    out = torch.empty_like(u) if out is None else _dev(out, "out")
    check(lib.nk_sh_residual(_ptr(u), _ptr(uo), _ptr(out), ny, nx, float(h), float(r), float(k),
                             float(g), _stream()), "nk_sh_residual")
    return out


def sh_jvp(u, v, h, r, k, g, ny=None, nx=None, out=None):
    """Exact J(u) v = v/k - (L v + (2 g u - 3 u^2) v)/2 of the residual above."""
    _dev(u, "u")
    _dev(v, "v")
    ny, nx = _grid(u, ny, nx)
    out = torch.empty_like(u) if out is None else _dev(out, "out")
    check(lib.nk_sh_jvp(_ptr(u), _ptr(v), _ptr(out), ny, nx, float(h), float(r), float(k),
                        float(g), _stream()), "nk_sh_jvp")
    return out


def sh_fdjvp(x0, G0, z, h, r, k, g, zs, sc, ny=None, nx=None, out=None):
    """FD matvec of KrylovJacobian (_nonlin.py:1500-1513): (G(x0 + sc*zs*z) - G0)/sc with
    G(w) = w/k - (L w + g w^2 - w^3)/2 (the x-dependent part of the residual)."""
    for t, nm in ((x0, "x0"), (G0, "G0"), (z, "z")):
        _dev(t, nm)
    ny, nx = _grid(x0, ny, nx)
    out = torch.empty_like(x0) if out is None else _dev(out, "out")
    check(lib.nk_sh_fdjvp(_ptr(x0), _ptr(G0), _ptr(z), _ptr(out), ny, nx, float(h), float(r),
                          float(k), float(g), float(zs), float(sc), _stream()), "nk_sh_fdjvp")
    return out


def sh_arnoldi_fused(V, coef, w, tau, x0, G0, h, r, k, g, zs, sc, z=None, ny=None, nx=None,
                     v_out=None, w_out=None, reduce=True, E=None, Ev_out=None, Ew_out=None):
    """One fused Arnoldi step (csrc/arnoldi.hip): the Gram-Schmidt update of scipy's _fgmres
    (_gcrotmk.py:104-143) ``v = tau*w + sum_i coef[i]*V[i]``, the next FD matvec
    (_nonlin.py:1500-1513) ``w' = (G(x0 + sc*zs*z) - G(x0))/sc`` with ``z = v`` unless given, and
    the next multi-dot, all in one pass over the basis.  Returns ``(v, w', dots)`` with
    ``dots = [w'.V_i..., w'.v, v.V_i..., v.v, w'.w']`` (None when ``reduce`` is False).  The
    difference quotient is evaluated in closed form, so ``G0`` is not read (it may be None).
    ``E`` (optional): the edge arrays (``edge_gather``) of V[0..nv-1] and w, from which the block
    halos are then read; ``Ev_out`` / ``Ew_out`` receive the edge arrays of v and w'."""
    for t, nm in ((w, "w"), (x0, "x0")):
        _dev(t, nm)
    ny, nx = _grid(x0, ny, nx)
    nv = len(V)
    ptrs = (C.c_void_p * max(nv, 1))(*[_dev(v, "V[i]").data_ptr() for v in V])
    cf = (C.c_double * max(nv, 1))(*[float(c) for c in coef])
    v_out = torch.empty_like(x0) if v_out is None else _dev(v_out, "v_out")
    w_out = torch.empty_like(x0) if w_out is None else _dev(w_out, "w_out")
    dots = (C.c_double * (2 * nv + 3))() if reduce else None
    zp = _ptr(_dev(z, "z")) if z is not None else None
    common = (cf, nv, _ptr(w), float(tau), _ptr(x0), _ptr(G0) if G0 is not None else None, zp,
              ny, nx, float(h), float(r), float(k), float(g), float(zs), float(sc), _ptr(v_out),
              _ptr(w_out))
    if E is None:
        check(lib.nk_sh_arnoldi_fused(ptrs, *common, dots, _stream()), "nk_sh_arnoldi_fused")
    else:
        if len(E) != nv + 1:
            raise ValueError("E holds the edge arrays of V[0..nv-1] and w")
        eptrs = (C.c_void_p * (nv + 1))(*[_dev(e, "E[i]").data_ptr() for e in E])
        check(lib.nk_sh_arnoldi_fused_edges(
            ptrs, eptrs, *common, _ptr(Ev_out) if Ev_out is not None else None,
            _ptr(Ew_out) if Ew_out is not None else None, dots, _stream()),
            "nk_sh_arnoldi_fused_edges")
    return v_out, w_out, (list(dots) if reduce else None)


def arnoldi_mbox_launches() -> int:
    """Fused Arnoldi launches (process-wide) whose block halos went through the mailbox
    (csrc/arnoldi.hip "Mailbox"; NKHIP_ARN_MBOX=0 turns it off)."""
    return int(lib.nk_arnoldi_mbox_launches())


def edge_gather(v, ny=None, nx=None, out=None):
    """The edge array of grid vector v (nkhip.h, nk_edge_gather): the two columns either side of
    every 256-column group boundary, four values per boundary and row."""
    _dev(v, "v")
    ny, nx = _grid(v, ny, nx)
    n = int(lib.nk_edge_elems(ny, nx))
    out = torch.empty(n, dtype=torch.float64, device=v.device) if out is None else out
    check(lib.nk_edge_gather(_ptr(v), _ptr(out), ny, nx, _stream()), "nk_edge_gather")
    return out


def dot(x, y) -> float:
    _dev(x, "x")
    _dev(y, "y")
    r = C.c_double()
    check(lib.nk_dot(_ptr(x), _ptr(y), x.numel(), C.byref(r), _stream()), "nk_dot")
    return r.value


def nrm2(x) -> float:
    _dev(x, "x")
    r = C.c_double()
    check(lib.nk_nrm2(_ptr(x), x.numel(), C.byref(r), _stream()), "nk_nrm2")
    return r.value


def maxnorm(x) -> float:
    """``np.absolute(x).max()`` (scipy/optimize/_nonlin.py:36-37)."""
    _dev(x, "x")
    r = C.c_double()
    check(lib.nk_maxnorm(_ptr(x), x.numel(), C.byref(r), _stream()), "nk_maxnorm")
    return r.value


def axpy(a, x, y):
    """y += a*x in place."""
    _dev(x, "x")
    _dev(y, "y")
    check(lib.nk_axpy(float(a), _ptr(x), _ptr(y), x.numel(), _stream()), "nk_axpy")
    return y


def scal(a, x):
    _dev(x, "x")
    check(lib.nk_scal(float(a), _ptr(x), x.numel(), _stream()), "nk_scal")
    return x


def mdot(V, w):
    """[v . w for v in V] in one pass over w."""
    _dev(w, "w")
    m = len(V)
    ptrs = (C.c_void_p * max(m, 1))(*[_dev(v, "V[i]").data_ptr() for v in V])
    out = (C.c_double * max(m, 1))()
    check(lib.nk_mdot(ptrs, m, _ptr(w), w.numel(), out, _stream()), "nk_mdot")
    return [out[i] for i in range(m)]


def maxpy(V, coef, y):
    """y += sum_i coef[i] * V[i] in one pass."""
    _dev(y, "y")
    m = len(V)
    ptrs = (C.c_void_p * max(m, 1))(*[_dev(v, "V[i]").data_ptr() for v in V])
    cs = (C.c_double * max(m, 1))(*[float(c) for c in coef])
    check(lib.nk_maxpy(ptrs, cs, m, _ptr(y), y.numel(), _stream()), "nk_maxpy")
    return y


def stream_copy(src, out=None):
    """out = src through nk_stream_copy (16-KB chunks per block, non-temporal): the bench's probe
    of the box's achievable streaming rate."""
    src = _dev(src, "src")
    out = torch.empty_like(src) if out is None else _dev(out, "out")
    if out.numel() != src.numel():
        raise ValueError("stream_copy: size mismatch")
    check(lib.nk_stream_copy(_ptr(src), _ptr(out), src.numel(), _stream()), "nk_stream_copy")
    return out
