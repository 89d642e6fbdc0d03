"""TEST INFRASTRUCTURE ONLY -- NumPy restatement of the droplet time-stepper (python_work/droplet.py).

Thin-film droplet coalescence h_t = div(h^3/3 grad p), p = -lap(h) + PI(h) + Bo cos(alpha) h, on a
91 x 61 moving mesh x = grad Q(xi, eta) (parabolic Monge-Ampere), Crank-Nicolson in time with
``newton_krylov(lambda u: residual(u, F, dt_n), U.val, maxiter=20, f_tol=1e-7)`` (droplet.py:383).

Layout: u[i*Nx + j], i = eta (row, Ny = 61), j = xi (column, Nx = 91) -- ``ksiksi`` comes from
``np.meshgrid`` (droplet.py:60), so x varies fastest.  Boundary index sets (make_Ibdy :762-776):
Left = column 0, Right = column Nx-1, Bottom = row 0, Top = row Ny-1.

Every function cites the reference lines it restates.  Reference quirks kept on purpose (SURVEY
8a row D2): compute_u_spatial_ders zeroes U_dksi[Bottom] where U_deta was probably meant (:722);
M.Leig is divided by dksi*deta (:833); A11/A22/A12 are recomputed from Q on every Laplace call
(:612-614, numerically the same as hoisting them per step, which the GPU path does).
"""
from __future__ import annotations

import math
from types import SimpleNamespace

import numpy as np

# -------------------------------------------------------------------- parameters (droplet.py:22-53)
P = SimpleNamespace(
    R=1.0, a=100.0, epsilon=1e-2, Nx=91, Ny=61, smoothing_iters=4,
    endl=-3.0, endr=6.0, endb=-3.0, endt=3.0,
    alpha=0.01, gamma=0.1, C=0.15,
    alpha2=0.0, n=6, m=3, Bo=0.01,
)  # a: droplet profile sharpness (:23)
P.a = 100.0
P.NN = P.Nx * P.Ny
P.Dx = P.endr - P.endl
P.Dy = P.endt - P.endb
P.dksi = P.Dx / (P.Nx - 1)
P.deta = P.Dy / (P.Ny - 1)
P.dksi2 = P.dksi * P.dksi
P.deta2 = P.deta * P.deta
P.epsilon2 = 1.0 / P.Dy

INIT_FILE = "initdrop_coal_1_91-61_100_0.01_0.01_0.1_0.15.txt"


# ---------------------------------------------------------------- 1-D operators (make_M :778-833)
def _d1_matrix(n, h):
    """dksiCentre / detaCentre 1-D factor (:795-806): 4th-order centred first derivative with
    one-sided closures on the two outer rows at each end."""
    A = np.zeros((n, n))
    for i in range(2, n - 2):
        A[i, i - 2:i + 3] = [1, -8, 0, 8, -1]
    A[0, :5] = [-25, 48, -36, 16, -3]
    A[1, :5] = [-3, -10, 18, -6, 1]
    A[-2, -5:] = [-1, 6, -18, 10, 3]
    A[-1, -5:] = [3, -16, 36, -48, 25]
    return A / (12 * h)


def _d2_matrix(n, h2):
    """d2ksi / d2eta 1-D factor (:782-793)."""
    A = np.zeros((n, n))
    for i in range(2, n - 2):
        A[i, i - 2:i + 3] = [-1, 16, -30, 16, -1]
    A[0, :5] = [-415 / 6, 96, -36, 32 / 3, -1.5]
    A[1, :6] = [10, -15, -4, 14, -6, 1]
    A[-1, -5:] = [-1.5, 32 / 3, -36, 96, -415 / 6]
    A[-2, -6:] = [1, -6, 14, -4, -15, 10]
    return A / (12 * h2)


D1X = _d1_matrix(P.Nx, P.dksi)
D1Y = _d1_matrix(P.Ny, P.deta)
D2X = _d2_matrix(P.Nx, P.dksi2)
D2Y = _d2_matrix(P.Ny, P.deta2)


def dksi(v):
    """M.dksiCentre.dot(v) = kron(I_y, D1x) v  (:800)."""
    return (v.reshape(P.Ny, P.Nx) @ D1X.T).reshape(-1)


def deta(v):
    """M.detaCentre.dot(v) = kron(D1y, I_x) v  (:805)."""
    return (D1Y @ v.reshape(P.Ny, P.Nx)).reshape(-1)


def d2ksi(v):
    return (v.reshape(P.Ny, P.Nx) @ D2X.T).reshape(-1)


def d2eta(v):
    return (D2Y @ v.reshape(P.Ny, P.Nx)).reshape(-1)


def dksideta(v):
    """M.dksideta = kron(D1y, D1x)  (:806)."""
    return (D1Y @ v.reshape(P.Ny, P.Nx) @ D1X.T).reshape(-1)


def _idx():
    I = np.arange(P.NN).reshape(P.Ny, P.Nx)
    return SimpleNamespace(Left=I[:, 0], Right=I[:, -1], Bottom=I[0, :], Top=I[-1, :],
                           Boundary=np.unique(np.concatenate([I[:, 0], I[:, -1], I[0, :], I[-1, :]])))


IB = _idx()


def leig():
    """M.Leig (:829-833), including the division by dksi*deta."""
    t = (2 * np.cos(np.pi * np.arange(P.Ny) / (P.Ny - 1)) - 2).reshape(P.Ny, 1) * np.ones(P.Nx) + \
        np.ones((P.Ny, 1)) * (2 * np.cos(np.pi * np.arange(P.Nx) / (P.Nx - 1)) - 2)
    return t / (P.dksi * P.deta)


# ------------------------------------------------------------------------------ mesh (Q) fields
def q_ders(qval):
    """compute_Q_spatial_ders (:696-711) + J (:376)."""
    Q = SimpleNamespace(val=qval)
    Q.dksi = dksi(qval)
    Q.deta = deta(qval)
    Q.dksi[IB.Left] = P.endl
    Q.dksi[IB.Right] = P.endr
    Q.deta[IB.Bottom] = P.endb
    Q.deta[IB.Top] = P.endt
    t = np.zeros(P.NN)
    t[IB.Left] = 25 / (6 * P.dksi) * abs(P.endl)
    t[IB.Right] = 25 / (6 * P.dksi) * abs(P.endr)
    Q.d2ksi = d2ksi(qval) + t
    t = np.zeros(P.NN)
    t[IB.Top] = 25 / (6 * P.deta) * abs(P.endt)
    t[IB.Bottom] = 25 / (6 * P.deta) * abs(P.endb)
    Q.d2eta = d2eta(qval) + t
    Q.dksideta = dksideta(qval)
    Q.dksideta[IB.Boundary] = 0
    Q.J = Q.d2ksi * Q.d2eta - Q.dksideta ** 2
    return Q


def metric(Q):
    """A11, A22, A12 of Laplace_operator (:612-614)."""
    A11 = (Q.dksideta ** 2 + Q.d2eta ** 2) / Q.J
    A22 = (Q.dksideta ** 2 + Q.d2ksi ** 2) / Q.J
    A12 = -(Q.dksideta * (Q.d2ksi + Q.d2eta)) / Q.J
    return A11, A22, A12


def laplace(v, v_dksi, v_deta, Q):
    """Laplace_operator (:601-681): J^-1 div_xi(J^-1 A grad_xi v) with the reference's explicit
    7-wide interior stencils, next-to and next-to-next-to boundary closures, and the cross terms."""
    A11f, A22f, A12 = metric(Q)
    A11 = A11f.reshape(P.Ny, P.Nx)
    A22 = A22f.reshape(P.Ny, P.Nx)
    v = v.reshape(P.Ny, P.Nx)
    vxx = np.zeros((P.Ny, P.Nx))
    vyy = np.zeros((P.Ny, P.Nx))
    dx2, dy2 = P.dksi2, P.deta2
    vxx[:, 3:-3] = (4 * A11[:, 2:-4] * (v[:, :-6] - 8 * v[:, 1:-5] + 8 * v[:, 3:-3] - v[:, 4:-2])
                    - (-A11[:, 1:-5] + 9 * A11[:, 2:-4] + 9 * A11[:, 3:-3] - A11[:, 4:-2])
                    * (v[:, 1:-5] - 27 * v[:, 2:-4] + 27 * v[:, 3:-3] - v[:, 4:-2])
                    + (-A11[:, 2:-4] + 9 * A11[:, 3:-3] + 9 * A11[:, 4:-2] - A11[:, 5:-1])
                    * (v[:, 2:-4] - 27 * v[:, 3:-3] + 27 * v[:, 4:-2] - v[:, 5:-1])
                    - 4 * A11[:, 4:-2] * (v[:, 2:-4] - 8 * v[:, 3:-3] + 8 * v[:, 5:-1] - v[:, 6:])) / (288 * dx2)
    vyy[3:-3, :] = (4 * A22[2:-4, :] * (v[:-6, :] - 8 * v[1:-5, :] + 8 * v[3:-3, :] - v[4:-2, :])
                    - (-A22[1:-5, :] + 9 * A22[2:-4, :] + 9 * A22[3:-3, :] - A22[4:-2, :])
                    * (v[1:-5, :] - 27 * v[2:-4, :] + 27 * v[3:-3, :] - v[4:-2, :])
                    + (-A22[2:-4, :] + 9 * A22[3:-3, :] + 9 * A22[4:-2, :] - A22[5:-1, :])
                    * (v[2:-4, :] - 27 * v[3:-3, :] + 27 * v[4:-2, :] - v[5:-1, :])
                    - 4 * A22[4:-2, :] * (v[2:-4, :] - 8 * v[3:-3, :] + 8 * v[5:-1, :] - v[6:, :])) / (288 * dy2)
    # next-to boundary
    vxx[:, 1] = A11[:, 1] * (10 * v[:, 0] - 15 * v[:, 1] - 4 * v[:, 2] + 14 * v[:, 3] - 6 * v[:, 4] + v[:, 5]) / (12 * dx2) \
        + (-3 * v[:, 0] - 10 * v[:, 1] + 18 * v[:, 2] - 6 * v[:, 3] + v[:, 4]) \
        * (-3 * A11[:, 0] - 10 * A11[:, 1] + 18 * A11[:, 2] - 6 * A11[:, 3] + A11[:, 4]) / (144 * dx2)
    vyy[1, :] = A22[1, :] * (10 * v[0, :] - 15 * v[1, :] - 4 * v[2, :] + 14 * v[3, :] - 6 * v[4, :] + v[5, :]) / (12 * dy2) \
        + (-3 * v[0, :] - 10 * v[1, :] + 18 * v[2, :] - 6 * v[3, :] + v[4, :]) \
        * (-3 * A22[0, :] - 10 * A22[1, :] + 18 * A22[2, :] - 6 * A22[3, :] + A22[4, :]) / (144 * dy2)
    vxx[:, -2] = A11[:, -2] * (10 * v[:, -1] - 15 * v[:, -2] - 4 * v[:, -3] + 14 * v[:, -4] - 6 * v[:, -5] + v[:, -6]) / (12 * dx2) \
        + (3 * v[:, -1] + 10 * v[:, -2] - 18 * v[:, -3] + 6 * v[:, -4] - v[:, -5]) \
        * (3 * A11[:, -1] + 10 * A11[:, -2] - 18 * A11[:, -3] + 6 * A11[:, -4] - A11[:, -5]) / (144 * dx2)
    vyy[-2, :] = A22[-2, :] * (10 * v[-1, :] - 15 * v[-2, :] - 4 * v[-3, :] + 14 * v[-4, :] - 6 * v[-5, :] + v[-6, :]) / (12 * dy2) \
        + (3 * v[-1, :] + 10 * v[-2, :] - 18 * v[-3, :] + 6 * v[-4, :] - v[-5, :]) \
        * (3 * A22[-1, :] + 10 * A22[-2, :] - 18 * A22[-3, :] + 6 * A22[-4, :] - A22[-5, :]) / (144 * dy2)
    # next-to-next-to boundary
    vxx[:, 2] = A11[:, 2] * (-v[:, 0] + 16 * v[:, 1] - 30 * v[:, 2] + 16 * v[:, 3] - v[:, 4]) / (12 * dx2) \
        + (v[:, 0] - 8 * v[:, 1] + 8 * v[:, 3] - v[:, 4]) * (A11[:, 0] - 8 * A11[:, 1] + 8 * A11[:, 3] - A11[:, 4]) / (144 * dx2)
    vyy[2, :] = A22[2, :] * (-v[0, :] + 16 * v[1, :] - 30 * v[2, :] + 16 * v[3, :] - v[4, :]) / (12 * dy2) \
        + (v[0, :] - 8 * v[1, :] + 8 * v[3, :] - v[4, :]) * (A22[0, :] - 8 * A22[1, :] + 8 * A22[3, :] - A22[4, :]) / (144 * dy2)
    vxx[:, -3] = A11[:, -3] * (-v[:, -1] + 16 * v[:, -2] - 30 * v[:, -3] + 16 * v[:, -4] - v[:, -5]) / (12 * dx2) \
        + (v[:, -5] - 8 * v[:, -4] + 8 * v[:, -2] - v[:, -1]) * (A11[:, -5] - 8 * A11[:, -4] + 8 * A11[:, -2] - A11[:, -1]) / (144 * dx2)
    vyy[-3, :] = A22[-3, :] * (-v[-1, :] + 16 * v[-2, :] - 30 * v[-3, :] + 16 * v[-4, :] - v[-5, :]) / (12 * dy2) \
        + (v[-5, :] - 8 * v[-4, :] + 8 * v[-2, :] - v[-1, :]) * (A22[-5, :] - 8 * A22[-4, :] + 8 * A22[-2, :] - A22[-1, :]) / (144 * dy2)
    # cross terms (A12 v_deta)_ksi, (A12 v_dksi)_eta
    t = dksi(A12 * v_deta)
    t[IB.Left] = 0
    t[IB.Right] = 0
    vxx = vxx.reshape(-1) + t
    t = deta(A12 * v_dksi)
    t[IB.Top] = 0
    t[IB.Bottom] = 0
    vyy = vyy.reshape(-1) + t
    return vxx / Q.J, vyy / Q.J


def PI(h):
    """Disjoining pressure (:462-467)."""
    n, m, eps = P.n, P.m, P.epsilon
    return (n - 1) * (m - 1) * ((eps / h) ** m - (eps / h) ** n) / (2 * eps * (n - m))


def pressure(h, hxx, hyy):
    """(:469-473)"""
    return -(hxx + hyy) + PI(h) + P.Bo * math.cos(P.alpha2) * h


def u_ders(uval, Q):
    """compute_u_spatial_ders (:713-727), with the U_dksi[Bottom] quirk (:722)."""
    U = SimpleNamespace(val=uval)
    ud = dksi(uval)
    ue = deta(uval)
    ud[IB.Left] = 0
    ud[IB.Right] = 0
    ue[IB.Top] = 0
    ud[IB.Bottom] = 0
    U.dx = (Q.d2eta * ud - Q.dksideta * ue) / Q.J
    U.dy = (-Q.dksideta * ud + Q.d2ksi * ue) / Q.J
    U.xx, U.yy = laplace(uval, ud, ue, Q)
    return U


def p_ders(pval, Q):
    """compute_P_spatial_ders (:683-694)."""
    pd = dksi(pval)
    pe = deta(pval)
    pd[IB.Left] = 0
    pd[IB.Right] = 0
    pe[IB.Top] = 0
    pe[IB.Bottom] = 0
    return (Q.d2eta * pd - Q.dksideta * pe) / Q.J, (-Q.dksideta * pd + Q.d2ksi * pe) / Q.J


def flux_div(h, pdx, pdy, Q):
    """pde_rhs (:452-460) / the F2 term of residual (:443-448)."""
    A = (pdx - P.Bo * math.sin(P.alpha2) / P.epsilon2) * (h ** 3) / 3
    B = pdy * (h ** 3) / 3
    return (Q.d2eta * dksi(A) - Q.dksideta * deta(A) - Q.dksideta * dksi(B) + Q.d2ksi * deta(B)) / Q.J


def step_rhs(uval, Q):
    """The old-time Crank-Nicolson term F of evolve_with_PDE (:374-381)."""
    U = u_ders(uval, Q)
    pval = pressure(uval, U.xx, U.yy)
    pdx, pdy = p_ders(pval, Q)
    return flux_div(uval, pdx, pdy, Q), U


def residual(u, F, dt, uval, Q):
    """residual(u, F, dt) (:435-450)."""
    uxx, uyy = laplace(u, dksi(u), deta(u), Q)
    pnew = pressure(u, uxx, uyy)
    pdx, pdy = p_ders(pnew, Q)
    F2 = flux_div(u, pdx, pdy, Q)
    return (u - uval) - dt * (F2 + F) / 2


# ------------------------------------------------------------------------------------- PMA
def monitor(U, Q):
    """compute_and_smooth_monitor (:729-760)."""
    temp = (np.abs(U.xx + U.yy) ** 2).reshape(P.Ny, P.Nx)
    Nx, Ny = P.Nx, P.Ny
    mon = np.zeros((Ny, Nx))
    for _ in range(P.smoothing_iters):
        mon[1:-1, 1:-1] = temp[1:-1, 1:-1] + (temp[:-2, 1:-1] + temp[2:, 1:-1] + temp[1:-1, :-2] + temp[1:-1, 2:]) / 8 \
            + (temp[:-2, :-2] + temp[:-2, 2:] + temp[2:, :-2] + temp[2:, 2:]) / 16
        mon[1:-1, Nx - 1] = (4 * temp[1:-1, Nx - 1] + 2 * temp[:-2, Nx - 1] + 2 * temp[2:, Nx - 1] + 2 * temp[1:-1, Nx - 2] + temp[2:, Nx - 2] + temp[:-2, Nx - 2]) / 12
        mon[1:-1, 0] = (4 * temp[1:-1, 0] + 2 * temp[:-2, 0] + 2 * temp[2:, 0] + 2 * temp[1:-1, 1] + temp[2:, 1] + temp[:-2, 1]) / 12
        mon[Ny - 1, 1:-1] = (4 * temp[Ny - 1, 1:-1] + 2 * temp[Ny - 1, :-2] + 2 * temp[Ny - 1, 2:] + 2 * temp[Ny - 2, 1:-1] + temp[Ny - 2, 2:] + temp[Ny - 2, :-2]) / 12
        mon[0, 1:-1] = (4 * temp[0, 1:-1] + 2 * temp[0, :-2] + 2 * temp[0, 2:] + 2 * temp[1, 1:-1] + temp[1, 2:] + temp[1, :-2]) / 12
        mon[0, 0] = (4 * temp[0, 0] + 2 * temp[0, 1] + 2 * temp[1, 0] + temp[1, 1]) / 9
        mon[0, Nx - 1] = (4 * temp[0, Nx - 1] + 2 * temp[0, Nx - 2] + 2 * temp[1, Nx - 1] + temp[1, Nx - 2]) / 9
        mon[Ny - 1, 0] = (4 * temp[Ny - 1, 0] + 2 * temp[Ny - 1, 1] + 2 * temp[Ny - 2, 0] + temp[Ny - 2, 1]) / 9
        mon[Ny - 1, Nx - 1] = (4 * temp[Ny - 1, Nx - 1] + 2 * temp[Ny - 1, Nx - 2] + 2 * temp[Ny - 2, Nx - 1] + temp[Ny - 2, Nx - 2]) / 9
        temp = mon.copy()
    mon = mon.reshape(-1)
    integ = np.sum(mon * np.abs(Q.J)) * P.dksi * P.deta
    return mon + P.C * integ


def solve_pma(U, Q, LEIG):
    """solve_PMA (:578-587): dQ/dt = (alpha (I - gamma Lap_xi))^-1 sqrt(M |J|) via 2-D DCT-II."""
    from scipy.fft import dct, idct
    mon = monitor(U, Q)
    q_rhs = np.sqrt(mon * np.abs(Q.J)) / P.alpha
    temp = dct(dct(q_rhs.reshape(P.Ny, P.Nx).T, norm="ortho").T, norm="ortho")
    dq = idct(idct((temp / (1 - P.gamma * LEIG)).T, norm="ortho").T, norm="ortho")
    return dq.reshape(-1)


def loop_pma(qval, uval, dtm, loops, Q=None, U=None):
    """loop_pma (:589-599).  Q/U: the derivative state already computed for the current Q (the
    first solve_PMA of the loop reuses the caller's U/Q/J, exactly like the reference)."""
    LEIG = leig()
    if Q is None:
        Q = q_ders(qval)
    if U is None:
        U = u_ders(uval, Q)
    qval = qval + dtm * solve_pma(U, Q, LEIG)
    for _ in range(1, loops):
        Q = q_ders(qval)
        U = u_ders(uval, Q)
        qval = qval + dtm * solve_pma(U, Q, LEIG)
    return qval


def evolve(uval, qval, nsteps, dt=1e-4, dtmesh=3e-9, pmaloops=400, newton=None, scale=1.0):
    """evolve_with_PDE (:360-411) without plotting: returns (U, Q, scale, dt list, nit list)."""
    if newton is None:
        from scipy.optimize import newton_krylov as newton
    u_new = uval.copy()
    dts = []
    for _ in range(nsteps):
        dt_n = dt * scale
        uval = u_new.copy()
        Q = q_ders(qval)
        F, U = step_rhs(uval, Q)
        u_new = newton(lambda u: residual(u, F, dt_n, uval, Q), uval, maxiter=20, f_tol=1e-7)
        qval = loop_pma(qval, uval, dtmesh, pmaloops, Q=Q, U=U)
        dts.append(dt_n)
        scale += np.exp(-10 * np.linalg.norm(u_new - uval))
    return u_new, qval, scale, dts


# ------------------------------------------------------------ initialisation (droplet.py:132-189)
def G2(xx, R):
    """(:425-426)"""
    return R + np.log((1 + np.exp(-2 * P.a * (xx + R))) / (1 + np.exp(-2 * P.a * (xx - R)))) / (2 * P.a)


def H2(psi, R, V):
    """(:428-429)"""
    return 4 * V * (1 - psi * psi / (R * R)) / (R * R)


def compute_U2(info, Q):
    """compute_U2 (:413-423): precursor film plus one parabolic cap per (x, y, R, V) droplet,
    evaluated at the physical node coordinates (Q.dksi, Q.deta)."""
    ret = np.full(P.NN, P.epsilon)
    for x, y, R, V in info:
        ret += (1 - P.epsilon) * H2(G2(np.sqrt((Q.dksi - x) ** 2 + (Q.deta - y) ** 2), R), R, V)
    return ret


def initial_mesh():
    """main() (:103): Q = (xi^2 + eta^2)/2, U = epsilon."""
    kk, ee = np.meshgrid(np.linspace(P.endl, P.endr, P.Nx), np.linspace(P.endb, P.endt, P.Ny))
    return np.full(P.NN, P.epsilon), np.reshape(0.5 * kk ** 2 + 0.5 * ee ** 2, P.NN)


def init_coalescing(vsteps=1000, info=((0, 0, 1, 1), (3, 0, 1, 1)), dtmesh=5e-9, loops=20,
                    unew=None, qval=None):
    """initialise_coalescing_droplets (:132-189) without plotting or file I/O: inflate the
    droplets' volumes linearly over `vsteps` steps, each followed by loop_pma(dtmesh, loops)."""
    if unew is None:
        unew, qval = initial_mesh()
    vf = [d[3] for d in info]
    for i in range(1, vsteps + 1):
        uval = unew.copy()
        Q = q_ders(qval)
        U = u_ders(uval, Q)
        arg = [(d[0], d[1], d[2], vf[k] * i / vsteps) for k, d in enumerate(info)]
        unew = compute_U2(arg, Q)
        qval = loop_pma(qval, uval, dtmesh, loops, Q=Q, U=U)
    return unew, qval
