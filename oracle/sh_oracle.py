"""TEST INFRASTRUCTURE ONLY -- NumPy restatement of the Swift-Hohenberg operators.

Restates ``/root/reference/python_work/sh_scipy_nk.py``:

* ``lap5``      -- periodic 5-point Laplacian ``Lap`` (sh_scipy_nk.py:32-35; C++ main.cpp:38-71).
                   Row-major flatten ``u[i*N + j]``: the N-sized diagonal blocks of ``Lap`` are
                   x-rows (sh_scipy_nk.py:34), the +-N diagonals couple y-neighbours (:35).
* ``sh13``      -- ``L = -Lap*Lap - 2*Lap + (r-1)*I`` (sh_scipy_nk.py:38-39; main.cpp:78-81)
                   applied matrix-free.  Closed-form 13-point coefficients from expanding
                   Lap^2 with ``Lap = e*(S - 4I)``:
                   centre -20e^2+8e+r-1, axial+-1 8e^2-2e, diagonal -2e^2, axial+-2 -e^2.
* ``residual``  -- the Crank-Nicolson residual (sh_scipy_nk.py:47-49; main.cpp:19-32), with the
                   reference's own association order (``L@u + g*uu - u*uu + L@Uo + g*UoUo - UoUoUo``).
* ``csr_L`` / ``scipy_sh_step`` -- the reference's CPU path as the reference runs it: an assembled
                   scipy CSR ``L`` (13 nnz/row) and ``scipy.optimize.newton_krylov(residual, Uo)``
                   (sh_scipy_nk.py:61).  This is the ``cpu_baseline`` leg of ``bench.py``.
"""
from __future__ import annotations

import numpy as np


def sh_coeffs(h: float, r: float):
    """13-point coefficients of L (sh_scipy_nk.py:38-39 with e = 1/h^2, :32)."""
    e = 1.0 / h ** 2
    c0 = -20.0 * e * e + 8.0 * e + r - 1.0
    c1 = 8.0 * e * e - 2.0 * e
    c2 = -2.0 * e * e
    c3 = -e * e
    return c0, c1, c2, c3


def _sh(v2, dy, dx):
    return np.roll(np.roll(v2, dy, axis=0), dx, axis=1)


def lap5(v: np.ndarray, ny: int, nx: int, e: float) -> np.ndarray:
    """``Lap @ v`` for the periodic 5-point Laplacian (sh_scipy_nk.py:32-35)."""
    v2 = np.asarray(v, dtype=np.float64).reshape(ny, nx)
    out = e * (_sh(v2, 1, 0) + _sh(v2, -1, 0) + _sh(v2, 0, 1) + _sh(v2, 0, -1) - 4.0 * v2)
    return out.reshape(-1)


def sh13(v: np.ndarray, ny: int, nx: int, h: float, r: float, dtype=np.float64) -> np.ndarray:
    """``L @ v`` with L = -Lap^2 - 2 Lap + (r-1) I (sh_scipy_nk.py:38-39), matrix-free."""
    c0, c1, c2, c3 = (dtype(c) for c in sh_coeffs(h, r))
    v2 = np.asarray(v, dtype=dtype).reshape(ny, nx)
    ax1 = _sh(v2, 1, 0) + _sh(v2, -1, 0) + _sh(v2, 0, 1) + _sh(v2, 0, -1)
    dg = _sh(v2, 1, 1) + _sh(v2, 1, -1) + _sh(v2, -1, 1) + _sh(v2, -1, -1)
    ax2 = _sh(v2, 2, 0) + _sh(v2, -2, 0) + _sh(v2, 0, 2) + _sh(v2, 0, -2)
    return (c0 * v2 + c1 * ax1 + c2 * dg + c3 * ax2).reshape(-1)


def residual(u, uo, ny, nx, h, r, k, g):
    """Crank-Nicolson residual F(u) of sh_scipy_nk.py:47-49 (C++ main.cpp:19-32)."""
    u = np.asarray(u, dtype=np.float64)
    uo = np.asarray(uo, dtype=np.float64)
    uu = u * u
    return (u - uo) / k - (sh13(u, ny, nx, h, r) + g * uu - u * uu
                           + sh13(uo, ny, nx, h, r) + g * (uo * uo) - uo * (uo * uo)) / 2


def jvp(u, v, ny, nx, h, r, k, g):
    """Exact Jacobian-vector product of ``residual`` at u: v/k - (Lv + (2g u - 3u^2) v)/2."""
    return v / k - (sh13(v, ny, nx, h, r) + (2.0 * g * u - 3.0 * u * u) * v) / 2


def fd_quotient(x0, u, alpha, sc, ny, nx, h, r, k, g, dtype=np.float64):
    """KrylovJacobian.matvec's difference quotient (_nonlin.py:1505-1509) on this residual,
    (F(x0 + alpha u) - F(x0)) / sc, evaluated with two residual evaluations (as SciPy does) in
    ``dtype``; F's constant part (the Uo terms) cancels, so G(w) = w/k - (Lw + g w^2 - w^3)/2."""
    x0 = np.asarray(x0, dtype=dtype)
    y = x0 + dtype(alpha) * np.asarray(u, dtype=dtype)

    def G(w):
        return w / dtype(k) - (sh13(w, ny, nx, h, r, dtype) + dtype(g) * w * w - w * w * w) / 2

    return (G(y) - G(x0)) / dtype(sc)


def fd_quotient_closed_form(x0, u, alpha, sc, ny, nx, h, r, k, g):
    """The same quotient in closed form (the fused Arnoldi kernel, csrc/arnoldi.hip): G is a
    cubic in w plus the linear stencil, so exactly
    (alpha/sc) [u/k - (L u + u (g (2 x0 + t) - (3 x0 (x0 + t) + t^2)))/2],  t = alpha u."""
    x0 = np.asarray(x0, dtype=np.float64)
    u = np.asarray(u, dtype=np.float64)
    t = alpha * u
    D = g * (2.0 * x0 + t) - (3.0 * x0 * (x0 + t) + t * t)
    return (alpha / sc) * (u / k - (sh13(u, ny, nx, h, r) + u * D) / 2)


# --------------------------------------------------------------------------------------
# The reference's CPU path (scipy CSR + scipy.optimize.newton_krylov): the CPU baseline.
# --------------------------------------------------------------------------------------

def csr_lap(n: int, h: float):
    """Assembled periodic 5-point Laplacian as the reference builds it (sh_scipy_nk.py:32-35):
    an N x N periodic tridiagonal block per x-row plus the +-N / +-(N^2-N) y-couplings."""
    import scipy.sparse as sp
    e = 1.0 / h ** 2
    ring = sp.diags([1.0, 1.0], [-1, 1], shape=(n, n), format="lil")
    ring[0, n - 1] = 1.0
    ring[n - 1, 0] = 1.0
    ring = ring.tocsr()
    eye = sp.identity(n, format="csr")
    return (e * (sp.kron(eye, ring) + sp.kron(ring, eye) - 4.0 * sp.identity(n * n))).tocsr()


def csr_L(n: int, h: float, r: float):
    """``L = -Lap*Lap - 2*Lap + (r-1)*I`` as an assembled CSR matrix (sh_scipy_nk.py:38-39)."""
    import scipy.sparse as sp
    lap = csr_lap(n, h)
    return (-(lap @ lap) - 2.0 * lap + (r - 1.0) * sp.identity(n * n, format="csr")).tocsr()


def make_csr_residual(L, uo, k, g, counter=None):
    """Closure with the reference's residual (sh_scipy_nk.py:47-49) over a CSR ``L``."""
    uo = np.asarray(uo, dtype=np.float64).copy()
    uouo = uo * uo
    uououo = uo * uouo

    def residual_fn(u):
        if counter is not None:
            counter[0] += 1
        uu = u * u
        return (u - uo) / k - (L @ u + g * uu - u * uu + L @ uo + g * uouo - uououo) / 2

    return residual_fn


def scipy_sh_step(L, uo, k, g, **nk_kwargs):
    """One implicit step exactly as the reference takes it (sh_scipy_nk.py:56-61)."""
    from scipy.optimize import newton_krylov
    cnt = [0]
    f = make_csr_residual(L, uo, k, g, cnt)
    u = newton_krylov(f, np.asarray(uo, dtype=np.float64), **nk_kwargs)
    return u, cnt[0]
