"""TEST INFRASTRUCTURE ONLY -- NumPy restatement of SciPy 1.15.3's ``newton_krylov`` stack.

The reference (``python_work/sh_scipy_nk.py:61``, ``PMA2_nk.py:100``, ``droplet.py:383``) calls the
third-party ``scipy.optimize.newton_krylov``; SciPy is not vendored in ``/root/reference`` and the
container's SciPy 1.15.3 is the de-facto pin.  This file restates its published algorithm:

* ``nonlin_solve``            scipy/optimize/_nonlin.py:122-268 (inexact Newton, Eisenstat-Walker
                              forcing gamma=0.9, eta_max=0.9999, threshold=0.1, eta0=1e-3)
* ``_line_search_armijo``     scipy/optimize/_nonlin.py:272-314 + _linesearch.py:684-739
* ``TerminationCondition``    scipy/optimize/_nonlin.py:317-375 (max-norm, f_tol = eps^(1/3))
* ``KrylovJacobian``          scipy/optimize/_nonlin.py:1453-1540 (FD JVP, omega update)
* ``lgmres`` (maxiter=1)      scipy/sparse/linalg/_isolve/lgmres.py:120-230
* ``_fgmres``                 scipy/sparse/linalg/_isolve/_gcrotmk.py:14-180 (MGS Arnoldi,
                              prepend_outer_v augmentation).  The Hessenberg QR of ``qr_insert`` is
                              restated with Givens rotations: ``res = |Q[0,-1]|`` is the last entry of
                              the rotated right-hand side, and ``lstsq(R, Q[0])`` is back-substitution.

``ortho="icwy"`` swaps MGS for the inverse-compact-WY form of MGS (one fused multi-dot + one
update per Arnoldi step) that the HIP solver uses; it is equal to MGS in exact arithmetic and
exists here only so that the CPU tests can show the two agree on the SH problem.
``ortho="lag"`` is icwy with the HIP solver's lagged norm (csrc/lgmres.cpp): the JVP of a new
basis vector is applied to ``v_raw / sqrt(|w|^2 - |h|^2)`` (norm 1 up to rounding, the FD step
taken as ``omega``) and rescaled once the exact norm is known.
"""
from __future__ import annotations

import math
import sys

import numpy as np

EPS = np.finfo(np.float64).eps


class NoConvergence(Exception):
    """Mirror of scipy.optimize.NoConvergence (_nonlin.py:30-33)."""


def maxnorm(x):
    return float(np.abs(x).max())


def _norm(x):
    return float(np.linalg.norm(x))


def _safe_norm(v):
    if not np.isfinite(v).all():
        return math.inf
    return _norm(v)


class _Stats:
    def __init__(self):
        self.nfev = 0
        self.njvp = 0
        self.nit = 0
        self.arnoldi = 0
        self.steps = []  # accepted line-search step s per Newton iteration


def _givens(a, b):
    if b == 0.0:
        return 1.0, 0.0
    rr = math.hypot(a, b)
    return a / rr, b / rr


def _lstsq_upper(R, g):
    """Least-squares solve of the (j+1)x(j+1) upper-triangular system (lstsq in _gcrotmk.py:177)."""
    n = R.shape[0]
    d = np.abs(np.diag(R))
    if n and d.min() > EPS * n * d.max():
        y = np.zeros(n)
        for i in range(n - 1, -1, -1):
            y[i] = (g[i] - R[i, i + 1:] @ y[i + 1:]) / R[i, i]
        return y
    return np.linalg.lstsq(R, g, rcond=None)[0]


def fgmres(matvec, v0, m, atol, outer_v, stats, ortho="mgs"):
    """_fgmres with prepend_outer_v=True, no preconditioner (_gcrotmk.py:14-180)."""
    vs = [v0]
    zs = []
    n_outer = len(outer_v)
    m = m + n_outer
    # Givens-QR of the Hessenberg matrix
    Rm = np.zeros((m + 1, m))
    cs = np.zeros(m)
    sn = np.zeros(m)
    gvec = np.zeros(m + 1)
    gvec[0] = 1.0
    gram = np.zeros((m + 1, m + 1))  # lower triangle v_i . v_k (icwy only)
    breakdown = False
    res = math.nan
    j = 0
    est = -1.0  # lag: |w|^2 - |h|^2 of the previous step
    wraw = None
    for j in range(m):
        if j < n_outer:
            z = outer_v[j]
        elif j == n_outer:
            z = v0
        else:
            z = vs[-1]
        if ortho == "lag" and j > n_outer and est > 1e-12 * wwprev:
            e = math.sqrt(est)
            w = (e / hprev) * matvec(wraw / e, unit=True)
        else:
            w = matvec(z)
        stats.arnoldi += 1
        w_norm = _norm(w)
        hcur = np.zeros(j + 2)
        if ortho == "mgs":
            for i, v in enumerate(vs):
                alpha = float(v @ w)
                hcur[i] = alpha
                w = w - alpha * v
        else:
            c = np.array([float(v @ w) for v in vs])
            for kk in range(j):
                gram[j, kk] = float(vs[j] @ vs[kk])
            h = np.zeros(j + 1)
            for i in range(j + 1):
                h[i] = c[i] - gram[i, :i] @ h[:i]
            hcur[:j + 1] = h
            w = w - sum(h[i] * vs[i] for i in range(j + 1))
            wwprev = w_norm * w_norm
            est = wwprev - float(h @ h)
            wraw = w
        hcur[j + 1] = _norm(w)
        hprev = hcur[j + 1]
        with np.errstate(over="ignore", divide="ignore"):
            alpha = 1.0 / hcur[-1]
        if np.isfinite(alpha):
            w = alpha * w
        if not (hcur[-1] > EPS * w_norm):
            breakdown = True
        vs.append(w)
        zs.append(z)
        # apply previous rotations, then a new one
        col = hcur.copy()
        for i in range(j):
            t = cs[i] * col[i] + sn[i] * col[i + 1]
            col[i + 1] = -sn[i] * col[i] + cs[i] * col[i + 1]
            col[i] = t
        cs[j], sn[j] = _givens(col[j], col[j + 1])
        col[j] = cs[j] * col[j] + sn[j] * col[j + 1]
        col[j + 1] = 0.0
        Rm[:j + 2, j] = col
        gvec[j + 1] = -sn[j] * gvec[j]
        gvec[j] = cs[j] * gvec[j]
        res = abs(gvec[j + 1])
        if res < atol or breakdown:
            break
    if not np.isfinite(Rm[j, j]):
        raise np.linalg.LinAlgError()
    y = _lstsq_upper(Rm[:j + 1, :j + 1], gvec[:j + 1])
    return vs, zs, y, res


class KrylovJacobian:
    """FD Krylov Jacobian (_nonlin.py:1453-1540) with lgmres, outer_k=10, inner_m=30."""

    def __init__(self, func, x, f, stats, rdiff=None, inner_m=30, outer_k=10, ortho="mgs"):
        self.func = func
        self.stats = stats
        self.rdiff = EPS ** 0.5 if rdiff is None else rdiff
        self.inner_m = inner_m
        self.outer_k = outer_k
        self.outer_v = []
        self.ortho = ortho
        self.update(x, f)

    def update(self, x, f):
        self.x0 = x
        self.f0 = f
        self.omega = self.rdiff * max(1.0, maxnorm(x)) / max(1.0, maxnorm(f))

    def matvec(self, v, unit=False):
        nv = 1.0 if unit else _norm(v)
        if nv == 0:
            return 0 * v
        sc = self.omega / nv
        r = (self.func(self.x0 + sc * v) - self.f0) / sc
        self.stats.njvp += 1
        if not np.all(np.isfinite(r)) and np.all(np.isfinite(v)):
            raise ValueError("Function returned non-finite results")
        return r

    def solve(self, b, tol):
        """lgmres(op, b, rtol=tol, atol=0, maxiter=1, ...) (lgmres.py:120-230)."""
        b_norm = _norm(b)
        if b_norm == 0:
            return b.copy()
        atol = max(0.0, tol * b_norm)
        r_norm = b_norm  # r_outer = matvec(0) - b = -b
        if r_norm <= max(atol, tol * b_norm):
            return np.zeros_like(b)
        v0 = b / b_norm
        inner_res_0 = b_norm
        ptol = min(1.0, max(atol, tol * b_norm) / r_norm)
        try:
            vs, zs, y, pres = fgmres(self.matvec, v0, self.inner_m, ptol, self.outer_v,
                                     self.stats, self.ortho)
            y = y * inner_res_0
            if not np.isfinite(y).all():
                raise np.linalg.LinAlgError()
        except np.linalg.LinAlgError:
            return np.zeros_like(b)
        dx = zs[0] * y[0]
        for w, yc in zip(zs[1:], y[1:]):
            dx = dx + yc * w
        nx = _norm(dx)
        if nx > 0:
            self.outer_v.append(dx / nx)
        while len(self.outer_v) > self.outer_k:
            del self.outer_v[0]
        return dx


def _armijo(phi, phi0, derphi0, c1=1e-4, alpha0=1.0, amin=0.0):
    """scalar_search_armijo (_linesearch.py:684-739)."""
    phi_a0 = phi(alpha0)
    if phi_a0 <= phi0 + c1 * alpha0 * derphi0:
        return alpha0, phi_a0
    alpha1 = -(derphi0) * alpha0 ** 2 / 2.0 / (phi_a0 - phi0 - derphi0 * alpha0)
    phi_a1 = phi(alpha1)
    if phi_a1 <= phi0 + c1 * alpha1 * derphi0:
        return alpha1, phi_a1
    while alpha1 > amin:
        factor = alpha0 ** 2 * alpha1 ** 2 * (alpha1 - alpha0)
        a = alpha0 ** 2 * (phi_a1 - phi0 - derphi0 * alpha1) - alpha1 ** 2 * (phi_a0 - phi0 - derphi0 * alpha0)
        a = a / factor
        b = -alpha0 ** 3 * (phi_a1 - phi0 - derphi0 * alpha1) + alpha1 ** 3 * (phi_a0 - phi0 - derphi0 * alpha0)
        b = b / factor
        alpha2 = (-b + np.sqrt(abs(b ** 2 - 3 * a * derphi0))) / (3.0 * a)
        phi_a2 = phi(alpha2)
        if phi_a2 <= phi0 + c1 * alpha2 * derphi0:
            return alpha2, phi_a2
        if (alpha1 - alpha2) > alpha1 / 2.0 or (1 - alpha2 / alpha1) < 0.96:
            alpha2 = alpha1 / 2.0
        alpha0, alpha1 = alpha1, alpha2
        phi_a0, phi_a1 = phi_a1, phi_a2
    return None, phi_a1


def _line_search(func, x, Fx, dx, smin=1e-2):
    """_nonlin_line_search with search_type='armijo' (_nonlin.py:272-314)."""
    tmp = {"s": 0.0, "phi": _norm(Fx) ** 2, "Fx": Fx}

    def phi(s):
        if s == tmp["s"]:
            return tmp["phi"]
        v = func(x + s * dx)
        p = _safe_norm(v) ** 2
        tmp.update(s=s, phi=p, Fx=v)
        return p

    s, _ = _armijo(phi, tmp["phi"], -tmp["phi"], amin=smin)
    if s is None:
        s = 1.0
    x = x + s * dx
    Fx = tmp["Fx"] if s == tmp["s"] else func(x)
    return s, x, Fx, _norm(Fx)


def newton_krylov(F, xin, *, rdiff=None, inner_m=30, outer_k=10, verbose=False, maxiter=None,
                  f_tol=None, f_rtol=None, x_tol=None, x_rtol=None, line_search="armijo",
                  ortho="mgs", return_stats=False):
    """nonlin_solve(F, xin, KrylovJacobian(...)) with SciPy defaults (_nonlin.py:122-268)."""
    stats = _Stats()
    f_tol = EPS ** (1.0 / 3) if f_tol is None else f_tol
    f_rtol = math.inf if f_rtol is None else f_rtol
    x_tol = math.inf if x_tol is None else x_tol
    x_rtol = math.inf if x_rtol is None else x_rtol
    x0 = np.asarray(xin, dtype=np.float64)

    def func(z):
        stats.nfev += 1
        return np.asarray(F(z.reshape(x0.shape)), dtype=np.float64).reshape(-1)

    x = x0.reshape(-1).copy()
    dx = np.full_like(x, np.inf)
    Fx = func(x)
    Fx_norm = _norm(Fx)
    jac = KrylovJacobian(func, x.copy(), Fx, stats, rdiff=rdiff, inner_m=inner_m,
                         outer_k=outer_k, ortho=ortho)
    if maxiter is None:
        maxiter = 100 * (x.size + 1)
    gamma, eta_max, eta_treshold, eta = 0.9, 0.9999, 0.1, 1e-3
    f0_norm = None
    converged = False
    for n in range(maxiter):
        stats.nit = n
        f_norm = maxnorm(Fx)
        if f0_norm is None:
            f0_norm = f_norm
        if f_norm == 0 or ((f_norm <= f_tol and f_norm / f_rtol <= f0_norm)
                           and (maxnorm(dx) <= x_tol and maxnorm(dx) / x_rtol <= maxnorm(x))):
            converged = True
            break
        tol = min(eta, eta * Fx_norm)
        dx = -jac.solve(Fx, tol)
        if _norm(dx) == 0:
            raise ValueError("Jacobian inversion yielded zero vector. "
                             "This indicates a bug in the Jacobian approximation.")
        if line_search:
            s, x, Fx, Fx_norm_new = _line_search(func, x, Fx, dx)
        else:
            s = 1.0
            x = x + dx
            Fx = func(x)
            Fx_norm_new = _norm(Fx)
        stats.steps.append(s)
        jac.update(x.copy(), Fx)
        eta_A = gamma * Fx_norm_new ** 2 / Fx_norm ** 2
        if gamma * eta ** 2 < eta_treshold:
            eta = min(eta_max, eta_A)
        else:
            eta = min(eta_max, max(eta_A, gamma * eta ** 2))
        Fx_norm = Fx_norm_new
        if verbose:
            sys.stdout.write("%d:  |F(x)| = %g; step %g\n" % (n, maxnorm(Fx), s))
    if not converged:
        stats.nit = maxiter
        raise NoConvergence(x.reshape(x0.shape))
    out = x.reshape(x0.shape)
    if return_stats:
        return out, stats
    return out
