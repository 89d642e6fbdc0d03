"""CPU: pin the PMA2 oracle (NumPy restatement of python_work/PMA2_nk.py) to the reference's own
outputs (tests/golden/make_golden_pma2.py: the reference module driven through main()'s loop body).

Tolerances (fp64): derived fields <= 1e-11 relative except Q_dksideta, which is ~1e-14 for the
paraboloid mesh and is compared absolutely; Newton-Krylov steps with the same iteration and
F-evaluation counts and |dU| <= 1e-12.
"""
import numpy as np

from conftest import load_golden
from oracle import nk_oracle
from oracle import pma2_oracle as O


def _rel(a, b):
    return float(np.abs(a - b).max() / max(np.abs(b).max(), 1e-300))


def test_fields_and_residual():
    f = load_golden("pma2_fields")
    Q = O.q_ders(f["Q_val"])
    U = O.u_ders(f["U_val"], Q)
    for key, val in [("Q_dksi", Q.dksi), ("Q_deta", Q.deta), ("Q_d2ksi", Q.d2ksi),
                     ("Q_d2eta", Q.d2eta), ("J", Q.J), ("U_dx", U.dx), ("U_dy", U.dy),
                     ("U_xx", U.xx), ("U_yy", U.yy)]:
        assert _rel(val, f[key]) <= 1e-11, key
    assert np.abs(Q.dksideta - f["Q_dksideta"]).max() <= 1e-20 + 1e-12 * np.abs(Q.d2ksi).max()
    assert _rel(O.monitor(U, Q), f["mon"]) <= 1e-13
    assert _rel(O.solve_pma(U, Q), f["Q_dt"]) <= 1e-13
    cn = O.new_rhs(f["U_val"], Q)
    assert _rel(cn, f["CN"]) <= 1e-11
    assert _rel(O.residual(f["u1"], f["U_val"], cn, Q), f["R1"]) <= 1e-11
    assert O.compute_g(f["U_val"]) * O.P.k == float(f["dt"])


def test_steps():
    s = load_golden("pma2_steps")
    u, q = s["U0"], s["Q0"]
    u0, q0 = O.initial_state()
    assert np.array_equal(u0, u) and np.array_equal(q0, q)
    for i in range(len(s["dt"])):
        (u, st), q, dt = O.step(u, q, newton=lambda F, x0: nk_oracle.newton_krylov(
            F, x0, return_stats=True))
        assert np.abs(u - s["U_new"][i]).max() <= 1e-12
        assert _rel(q, s["Q_val"][i]) <= 1e-13
        assert abs(dt - s["dt"][i]) <= 1e-18
        assert st.nit == s["nit"][i] and st.nfev == s["nfev"][i]


def test_configure_other_grid_and_back():
    """configure(n) rebuilds every grid-dependent global (the GPU test of other grid sizes uses
    it); configure(51) restores the reference's grid exactly, so the fixture tests still hold."""
    D1, D2 = O.D1.copy(), O.D2.copy()
    try:
        O.configure(37)
        assert O.P.N == 37 and O.P.NN == 37 * 37 and O.D1.shape == (37, 37)
        assert O.IB.Boundary.size == 4 * 37 - 4
        u, q = O.initial_state()
        assert u.shape == q.shape == (37 * 37,)
        assert np.isfinite(O.solve_pma(O.u_ders(u, O.q_ders(q)), O.q_ders(q))).all()
    finally:
        O.configure(51)
    assert np.array_equal(O.D1, D1) and np.array_equal(O.D2, D2) and O.P.NN == 51 * 51
