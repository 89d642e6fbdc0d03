"""TEST INFRASTRUCTURE ONLY -- NumPy restatement of the MEMS moving-mesh stepper
(python_work/PMA2_nk.py).

    u_t = -(-Lap)^p u - lambda/(1+u)^2 + lambda eps^(m-2)/(1+u)^m      (p = 2 in the reference)

on an N x N mesh x = grad Q(xi, eta) over [-1, 1]^2 (N = 51), Crank-Nicolson in time through
``newton_krylov(residual, U.val, verbose=0)`` with SciPy defaults (:100), and ONE parabolic
Monge-Ampere mesh step per time step (solve_PMA before the solve, ``Q.val += dt*Q.dt`` after).

Layout: u[i*N + j], i = eta row, j = xi column (``np.meshgrid``, :43).  Quirks kept on purpose
(SURVEY 8a row D3): residual() divides by the module-global dt = k (:51) because main() only
assigns a local dt (:91); the adaptive dt = min((1+u)^3) k moves the mesh and the clock only.
The p == 1 branch of residual() reads ``u.xx`` and would raise (:135): only p = 2 is restated.
Every function cites the reference lines it restates.
"""
from __future__ import annotations

from types import SimpleNamespace

import numpy as np

from .droplet_oracle import _d1_matrix, _d2_matrix

# ---------------------------------------------------------------- parameters (PMA2_nk.py:22-40)
P = SimpleNamespace(N=51, p=2, m=3, alpha=0.1, gamma=0.1, epsilon=0.0, beta=0.15,
                    smoothing_iters=4, lambd=1.0, endl=-1.0, endr=1.0, k=1e-4, Tf=0.3)
P.NN = P.N * P.N
P.d = P.endr - P.endl
P.dksi = P.d / (P.N - 1)
P.dksi2 = P.dksi * P.dksi


def configure(n):
    """The grid-dependent globals for an n x n grid (the reference's N = 51; other sizes exercise
    the GPU path's even / odd DCT split on both parities of N)."""
    global D1, D2, _I, IB
    P.N = n
    P.NN = n * n
    P.dksi = P.d / (n - 1)
    P.dksi2 = P.dksi * P.dksi
    D1 = _d1_matrix(n, P.dksi)    # A.2 (:195-201)
    D2 = _d2_matrix(n, P.dksi2)   # A.1 (:184-193)
    _I = np.arange(P.NN).reshape(n, n)
    IB = SimpleNamespace(Left=_I[:, 0], Right=_I[:, -1], Bottom=_I[0, :], Top=_I[-1, :])
    IB.Boundary = np.unique(np.concatenate([IB.Left, IB.Right, IB.Bottom, IB.Top]))  # make_Ibdy (:164-178)


configure(P.N)


def dksi(v):
    """M.dksiCentre = kron(eye, D1) (:200)."""
    return (v.reshape(P.N, P.N) @ D1.T).reshape(-1)


def deta(v):
    """M.detaCentre = kron(D1, eye) (:201)."""
    return (D1 @ v.reshape(P.N, P.N)).reshape(-1)


def initial_state():
    """main() initialisation (:65-71): Q = (xi^2 + eta^2)/2, U = 0."""
    ksi = np.linspace(P.endl, P.endr, P.N)
    kk, ee = np.meshgrid(ksi, ksi)
    return np.zeros(P.NN), np.reshape(0.5 * kk ** 2 + 0.5 * ee ** 2, P.NN)


def leig():
    """M.Leig (:228-231)."""
    c = 2 * np.cos(np.pi * np.arange(P.N) / (P.N - 1)) - 2
    return (c.reshape(P.N, 1) * np.ones(P.N) + np.ones((P.N, 1)) * c) / P.dksi2


def q_ders(qval):
    """compute_Q_spatial_ders (:233-249) + J (:84)."""
    Q = SimpleNamespace(val=qval)
    Q.dksi = dksi(qval)
    Q.dksi[IB.Left] = -1
    Q.dksi[IB.Right] = 1
    Q.deta = deta(qval)
    Q.deta[IB.Bottom] = -1
    Q.deta[IB.Top] = 1
    extra = 25 / (6 * P.dksi)
    t = np.zeros(P.NN)
    t[IB.Left] = extra
    t[IB.Right] = extra
    Q.d2ksi = (qval.reshape(P.N, P.N) @ D2.T).reshape(-1) + t
    t = np.zeros(P.NN)
    t[IB.Top] = extra
    t[IB.Bottom] = extra
    Q.d2eta = (D2 @ qval.reshape(P.N, P.N)).reshape(-1) + t
    Q.dksideta = (D1 @ qval.reshape(P.N, P.N) @ D1.T).reshape(-1)   # kron(D1, D1) (:202)
    Q.dksideta[IB.Boundary] = 0
    Q.J = Q.d2ksi * Q.d2eta - Q.dksideta ** 2
    return Q


def laplace(v, v_dksi, v_deta, Q):
    """Laplace_operator (:263-343), the same discretisation as droplet.py's."""
    n, h2 = P.N, P.dksi2
    A11 = ((Q.dksideta ** 2 + Q.d2eta ** 2) / Q.J).reshape(n, n)
    A22 = ((Q.dksideta ** 2 + Q.d2ksi ** 2) / Q.J).reshape(n, n)
    A12 = -(Q.dksideta * (Q.d2ksi + Q.d2eta)) / Q.J
    v = v.reshape(n, n)

    def axis(w, a):
        """B.1 along the last axis of w (rows = independent lines)."""
        out = np.zeros_like(w)
        out[:, 3:-3] = (4 * a[:, 2:-4] * (w[:, :-6] - 8 * w[:, 1:-5] + 8 * w[:, 3:-3] - w[:, 4:-2])
                        - (-a[:, 1:-5] + 9 * a[:, 2:-4] + 9 * a[:, 3:-3] - a[:, 4:-2])
                        * (w[:, 1:-5] - 27 * w[:, 2:-4] + 27 * w[:, 3:-3] - w[:, 4:-2])
                        + (-a[:, 2:-4] + 9 * a[:, 3:-3] + 9 * a[:, 4:-2] - a[:, 5:-1])
                        * (w[:, 2:-4] - 27 * w[:, 3:-3] + 27 * w[:, 4:-2] - w[:, 5:-1])
                        - 4 * a[:, 4:-2] * (w[:, 2:-4] - 8 * w[:, 3:-3] + 8 * w[:, 5:-1] - w[:, 6:])) / (288 * h2)
        out[:, 1] = a[:, 1] * (10 * w[:, 0] - 15 * w[:, 1] - 4 * w[:, 2] + 14 * w[:, 3] - 6 * w[:, 4] + w[:, 5]) / (12 * h2) \
            + (-3 * w[:, 0] - 10 * w[:, 1] + 18 * w[:, 2] - 6 * w[:, 3] + w[:, 4]) \
            * (-3 * a[:, 0] - 10 * a[:, 1] + 18 * a[:, 2] - 6 * a[:, 3] + a[:, 4]) / (144 * h2)
        out[:, -2] = a[:, -2] * (10 * w[:, -1] - 15 * w[:, -2] - 4 * w[:, -3] + 14 * w[:, -4] - 6 * w[:, -5] + w[:, -6]) / (12 * h2) \
            + (3 * w[:, -1] + 10 * w[:, -2] - 18 * w[:, -3] + 6 * w[:, -4] - w[:, -5]) \
            * (3 * a[:, -1] + 10 * a[:, -2] - 18 * a[:, -3] + 6 * a[:, -4] - a[:, -5]) / (144 * h2)
        out[:, 2] = a[:, 2] * (-w[:, 0] + 16 * w[:, 1] - 30 * w[:, 2] + 16 * w[:, 3] - w[:, 4]) / (12 * h2) \
            + (w[:, 0] - 8 * w[:, 1] + 8 * w[:, 3] - w[:, 4]) * (a[:, 0] - 8 * a[:, 1] + 8 * a[:, 3] - a[:, 4]) / (144 * h2)
        out[:, -3] = a[:, -3] * (-w[:, -1] + 16 * w[:, -2] - 30 * w[:, -3] + 16 * w[:, -4] - w[:, -5]) / (12 * h2) \
            + (w[:, -5] - 8 * w[:, -4] + 8 * w[:, -2] - w[:, -1]) * (a[:, -5] - 8 * a[:, -4] + 8 * a[:, -2] - a[:, -1]) / (144 * h2)
        return out

    vxx = axis(v, A11).reshape(-1)
    vyy = axis(v.T, A22.T).T.reshape(-1)
    t = dksi(A12 * v_deta)          # B.2 (:332-342)
    t[IB.Left] = 0
    t[IB.Right] = 0
    vxx = vxx + t
    t = deta(A12 * v_dksi)
    t[IB.Top] = 0
    t[IB.Bottom] = 0
    vyy = vyy + t
    return vxx / Q.J, vyy / Q.J


def new_rhs(u, Q):
    """The right-hand side of residual() (:132-157) = compute_rhs_pde() at u (:400-413):
    -lambda/(1+u)^2 + lambda eps^(m-2)/(1+u)^m - beta^2 Lap(Lap u), zero on the boundary."""
    r = -P.lambd / ((1 + u) ** 2) + P.lambd * (P.epsilon ** (P.m - 2)) / ((1 + u) ** P.m)
    uxx, uyy = laplace(u, dksi(u), deta(u), Q)
    v = uxx + uyy
    vxx, vyy = laplace(v, dksi(v), deta(v), Q)
    r = r - P.beta * P.beta * (vxx + vyy)
    r[IB.Boundary] = 0
    return r


def residual(u, uval, cn, Q):
    """residual(u) (:121-159) with the global dt = k (quirk, :51/:91)."""
    return (u - uval) / P.k - (new_rhs(u, Q) + cn) / 2


def u_ders(uval, Q):
    """compute_u_spatial_ders (:251-261): raw derivatives, no boundary rules."""
    U = SimpleNamespace(val=uval)
    ud, ue = dksi(uval), deta(uval)
    U.dx = (Q.d2eta * ud - Q.dksideta * ue) / Q.J
    U.dy = (-Q.dksideta * ud + Q.d2ksi * ue) / Q.J
    U.xx, U.yy = laplace(uval, ud, ue, Q)
    return U


def monitor(U, Q):
    """compute_and_smooth_monitor (:345-386): eps == 0 -> 1/(1+u)^6; p == 2 -> |u_xx + u_yy|^2."""
    n = P.N
    if P.epsilon == 0:
        temp = (1 / (1 + U.val) ** 6).reshape(n, n)
    elif P.p == 1:
        temp = (1 + U.dx ** 2 + U.dy ** 2).reshape(n, n)
    else:
        temp = (np.abs(U.xx + U.yy) ** 2).reshape(n, n)
    mon = np.zeros((n, n))
    for _ in range(P.smoothing_iters):
        mon[1:-1, 1:-1] = temp[1:-1, 1:-1] + (temp[:-2, 1:-1] + temp[2:, 1:-1] + temp[1:-1, :-2] + temp[1:-1, 2:]) / 8 \
            + (temp[:-2, :-2] + temp[:-2, 2:] + temp[2:, :-2] + temp[2:, 2:]) / 16
        mon[1:-1, n - 1] = (4 * temp[1:-1, n - 1] + 2 * temp[:-2, n - 1] + 2 * temp[2:, n - 1] + 2 * temp[1:-1, n - 2] + temp[2:, n - 2] + temp[:-2, n - 2]) / 12
        mon[1:-1, 0] = (4 * temp[1:-1, 0] + 2 * temp[:-2, 0] + 2 * temp[2:, 0] + 2 * temp[1:-1, 1] + temp[2:, 1] + temp[:-2, 1]) / 12
        mon[n - 1, 1:-1] = (4 * temp[n - 1, 1:-1] + 2 * temp[n - 1, :-2] + 2 * temp[n - 1, 2:] + 2 * temp[n - 2, 1:-1] + temp[n - 2, 2:] + temp[n - 2, :-2]) / 12
        mon[0, 1:-1] = (4 * temp[0, 1:-1] + 2 * temp[0, :-2] + 2 * temp[0, 2:] + 2 * temp[1, 1:-1] + temp[1, 2:] + temp[1, :-2]) / 12
        mon[0, 0] = (4 * temp[0, 0] + 2 * temp[0, 1] + 2 * temp[1, 0] + temp[1, 1]) / 9
        mon[0, n - 1] = (4 * temp[0, n - 1] + 2 * temp[0, n - 2] + 2 * temp[1, n - 1] + temp[1, n - 2]) / 9
        mon[n - 1, 0] = (4 * temp[n - 1, 0] + 2 * temp[n - 1, 1] + 2 * temp[n - 2, 0] + temp[n - 2, 1]) / 9
        mon[n - 1, n - 1] = (4 * temp[n - 1, n - 1] + 2 * temp[n - 1, n - 2] + 2 * temp[n - 2, n - 1] + temp[n - 2, n - 2]) / 9
        temp = mon.copy()
    mon = mon.reshape(-1)
    return mon + np.sum(mon * np.abs(Q.J)) * P.dksi2      # Mackenzie regularisation (:383-385)


def solve_pma(U, Q):
    """solve_PMA (:388-398)."""
    from scipy.fft import dct, idct
    q_rhs = np.sqrt(monitor(U, Q) * np.abs(Q.J)) / P.alpha
    temp = dct(dct(q_rhs.reshape(P.N, P.N).T, norm="ortho").T, norm="ortho")
    return idct(idct((temp / (1 - P.gamma * leig())).T, norm="ortho").T, norm="ortho").reshape(-1)


def compute_g(uval):
    """compute_g (:437-441)."""
    return np.min((1 + uval) ** 3) if P.epsilon == 0 else 1.0


def step(unew, qval, newton=None, **nk):
    """One pass of main()'s loop body (:77-106).  Returns (U.new, Q.val, dt)."""
    if newton is None:
        from scipy.optimize import newton_krylov as newton
    uval = unew.copy()
    Q = q_ders(qval)
    U = u_ders(uval, Q)
    dt = compute_g(uval) * P.k
    qdt = solve_pma(U, Q)
    cn = new_rhs(uval, Q)
    unew = newton(lambda u: residual(u, uval, cn, Q), uval, **nk)
    return unew, qval + dt * qdt, dt
