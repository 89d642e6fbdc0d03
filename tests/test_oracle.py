"""CPU: pin the oracle (NumPy restatement) against the reference's own golden vectors.

The fixtures were produced by executing the reference ``sh_scipy_nk.py`` prologue (lines 1-49)
and driving ``scipy.optimize.newton_krylov`` as its loop does (tests/golden/make_golden.py).
"""
import numpy as np
import pytest

from conftest import load_golden
from oracle import nk_oracle, sh_oracle

OPS = ["ops_n5_d2", "ops_n61", "ops_n64", "ops_n128_h0625"]


@pytest.mark.parametrize("name", OPS)
def test_stencils_match_reference_csr(name):
    z = load_golden(name)
    N, h, r = int(z["N"]), float(z["h"]), float(z["r"])
    v = z["v"]
    lap = sh_oracle.lap5(v, N, N, 1.0 / h ** 2)
    L = sh_oracle.sh13(v, N, N, h, r)
    assert np.abs(lap - z["lap_v"]).max() <= 1e-13 * np.abs(z["lap_v"]).max()
    assert np.abs(L - z["L_v"]).max() <= 1e-13 * np.abs(z["L_v"]).max()
    if N >= 5:
        assert int(z["L_nnz"]) == 13 * N * N  # 13-point operator (sh_scipy_nk.py:38-39)


@pytest.mark.parametrize("name", OPS)
def test_csr_restatement_matches_reference(name):
    z = load_golden(name)
    N, h, r = int(z["N"]), float(z["h"]), float(z["r"])
    L = sh_oracle.csr_L(N, h, r)
    assert L.nnz == int(z["L_nnz"])
    assert np.abs(L @ z["v"] - z["L_v"]).max() <= 1e-13 * np.abs(z["L_v"]).max()


def test_residual_matches_reference():
    z = load_golden("residual_n61")
    F = sh_oracle.residual(z["u"], z["uo"], 61, 61, float(z["h"]), float(z["r"]), float(z["k"]),
                           float(z["g"]))
    assert np.abs(F - z["F"]).max() <= 1e-12 * np.abs(z["F"]).max()


def test_jvp_is_derivative_of_residual():
    z = load_golden("residual_n61")
    h, r, k, g = float(z["h"]), float(z["r"]), float(z["k"]), float(z["g"])
    u, uo = z["u"], z["uo"]
    v = np.random.default_rng(3).standard_normal(u.size)
    eps = 1e-6
    fd = (sh_oracle.residual(u + eps * v, uo, 61, 61, h, r, k, g)
          - sh_oracle.residual(u - eps * v, uo, 61, 61, h, r, k, g)) / (2 * eps)
    J = sh_oracle.jvp(u, v, 61, 61, h, r, k, g)
    assert np.abs(J - fd).max() <= 1e-6 * np.abs(J).max()


NK = ["nk_n61_default", "nk_n61_tight", "nk_n64_default", "nk_n64_h0625_tight",
      "nk_n5_d2_tight", "nk_n61_amp3_backtrack"]


@pytest.mark.parametrize("name", NK)
@pytest.mark.parametrize("ortho", ["mgs", "icwy", "lag"])
def test_nk_restatement_matches_scipy_steps(name, ortho):
    z = load_golden(name)
    N, h, r, k, g = int(z["N"]), float(z["h"]), float(z["r"]), float(z["k"]), float(z["g"])
    ftol = None if np.isnan(z["f_tol"]) else float(z["f_tol"])
    traj = z["traj"]
    for s in range(len(traj) - 1):
        uo = traj[s]
        F = lambda u, uo=uo: sh_oracle.residual(u, uo, N, N, h, r, k, g)  # noqa: E731
        u, st = nk_oracle.newton_krylov(F, uo, f_tol=ftol, return_stats=True, ortho=ortho)
        ref = traj[s + 1]
        scale = max(1.0, np.abs(ref).max())
        tol = 1e-8 if ftol is not None else 1e-5
        assert np.abs(u - ref).max() <= tol * scale
        assert abs(st.nit - int(z["nit"][s])) <= 1
        if ortho == "mgs" and ftol is not None:
            assert st.nfev == int(z["nfev"][s])


def test_nk_restatement_raises_like_scipy():
    z = load_golden("nk_n61_default")
    N, h = 61, float(z["h"])
    uo = z["traj"][0]
    F = lambda u: sh_oracle.residual(u, uo, N, N, h, 0.01, 0.2, 1.0)  # noqa: E731
    with pytest.raises(nk_oracle.NoConvergence):
        nk_oracle.newton_krylov(F, uo, maxiter=1)


@pytest.mark.parametrize("alpha", [1e-8, 1e-4, 0.3])
def test_fd_quotient_closed_form(alpha):
    """The fused kernel's closed-form JVP equals SciPy's two-evaluation difference quotient: exactly
    in exact arithmetic, so against the quotient evaluated in extended precision it agrees to
    double rounding, while the float64 two-evaluation form carries its cancellation error
    ~eps |G| / (alpha |J u|) (largest at SciPy's tiny steps)."""
    N, h, r, k, g = 48, 0.625, 0.01, 0.2, 1.0
    rng = np.random.default_rng(5)
    x0 = rng.standard_normal(N * N)
    u = rng.standard_normal(N * N) / N
    sc = alpha / 0.5
    closed = sh_oracle.fd_quotient_closed_form(x0, u, alpha, sc, N, N, h, r, k, g)
    ext = sh_oracle.fd_quotient(x0, u, alpha, sc, N, N, h, r, k, g, dtype=np.longdouble)
    two = sh_oracle.fd_quotient(x0, u, alpha, sc, N, N, h, r, k, g)
    scale = float(np.abs(ext).max())
    err_closed = float(np.abs(closed - ext.astype(np.float64)).max()) / scale
    err_two = float(np.abs(two - ext.astype(np.float64)).max()) / scale
    # long double has 64-bit mantissa here; its own error is ~eps_ld |G| / (alpha |J u|)
    eps_ld = float(np.finfo(np.longdouble).eps)
    assert err_closed <= 1e-13 + 1e3 * eps_ld / alpha
    assert err_closed <= err_two + 1e-13
    # the two-evaluation form's error grows as the step shrinks; the closed form's does not
    if alpha <= 1e-4:
        assert err_two >= 10 * err_closed


def test_nk_restatement_backtracks_like_scipy():
    """a step whose Armijo search backtracks (s < 1, quadratic and cubic
    branches of scalar_search_armijo) -- the restatement takes scipy's step sizes and F evals."""
    z = load_golden("nk_n61_amp3_backtrack")
    N, h, r, k, g = int(z["N"]), float(z["h"]), float(z["r"]), float(z["k"]), float(z["g"])
    uo = z["traj"][0]
    F = lambda u: sh_oracle.residual(u, uo, N, N, h, r, k, g)  # noqa: E731
    u, st = nk_oracle.newton_krylov(F, uo, return_stats=True, ortho="mgs")
    ref = z["steps"]
    assert (ref < 1).sum() >= 4  # the fixture does backtrack
    # With eta ~ 0.9 forcing the inexact Newton directions carry the FD-JVP rounding noise, so
    # the accepted steps agree to ~1 % (not bitwise); the backtracking pattern is identical.
    assert st.nit == int(z["nit"][0])
    np.testing.assert_array_equal(np.array(st.steps) < 1, ref < 1)
    np.testing.assert_allclose(st.steps, ref, rtol=3e-2)
    assert abs(st.nfev - int(z["nfev"][0])) <= 0.03 * int(z["nfev"][0])
    assert np.abs(u - z["traj"][1]).max() <= 1e-5 * max(1.0, np.abs(z["traj"][1]).max())


def test_nk_restatement_tracks_reference_trajectory():
    """The time loop (sh_scipy_nk.py:53-61) at the reference defaults (N = 64, d = 40): the
    NumPy restatement of SciPy's newton_krylov, stepped 100 times from default_rng(2020), stays
    within 1e-7 of the reference's own trajectory at every 10th step (measured 9e-9 at step 100)
    with the same Newton count per step.  Pins tests/golden/nk_n64_traj100.npz."""
    z = load_golden("nk_n64_traj100")
    N, h, r, k, g = int(z["N"]), float(z["h"]), float(z["r"]), float(z["k"]), float(z["g"])
    U = z["traj"][0].copy()
    nits = []
    for s in range(1, int(z["steps"][-1]) + 1):
        uo = U.copy()
        F = lambda u: sh_oracle.residual(u, uo, N, N, h, r, k, g)  # noqa: E731
        U, st = nk_oracle.newton_krylov(F, uo, return_stats=True, ortho="mgs")
        nits.append(st.nit)
        if s % 10 == 0:
            ref = z["traj"][s // 10]
            assert np.abs(U - ref).max() <= 1e-7 * max(1.0, np.abs(ref).max()), s
    assert nits == [int(x) for x in z["nit"]]
