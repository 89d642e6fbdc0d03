"""GPU: the PMA2 MEMS stepper (python_work/PMA2_nk.py) against the reference's
outputs (tests/golden/make_golden_pma2.py).

Tolerances (fp64): mesh / Laplace fields <= 1e-10 relative (stencils vs the reference's sparse
products: different summation order); CN_term and the residual <= 1e-9 relative (two stacked
Laplace_operator applications amplify rounding by ~1/h^4); each Newton-Krylov step (SciPy
defaults, f_tol = eps^(1/3)) within 1e-9 absolute of the reference's U (|U| ~ 1e-4 here) with the
same Newton-iteration count; Q within 1e-12 relative.
"""
import numpy as np
import pytest
import torch

from conftest import load_golden

pytestmark = pytest.mark.gpu


def _rel(a, b):
    a = a.detach().cpu().numpy() if isinstance(a, torch.Tensor) else a
    return float(np.abs(a - b).max() / max(np.abs(b).max(), 1e-300))


@pytest.fixture
def mems():
    import nkhip
    m = nkhip.Mems()
    yield m
    m.close()


def test_initial_state(mems):
    s = load_golden("pma2_steps")
    U, Q = mems.state()
    assert np.array_equal(U.cpu().numpy(), s["U0"]) and np.array_equal(Q.cpu().numpy(), s["Q0"])


def test_fields_and_residual(mems):
    f = load_golden("pma2_fields")
    mems.set_state(f["U_val"], f["Q_val"])
    dt = mems.prepare()
    assert abs(dt - float(f["dt"])) <= 1e-18
    for name, key, tol in [("Q_dksi", "Q_dksi", 1e-13), ("Q_deta", "Q_deta", 1e-13),
                           ("d2ksi", "Q_d2ksi", 1e-10), ("d2eta", "Q_d2eta", 1e-10),
                           ("J", "J", 1e-10), ("U_xx", "U_xx", 1e-10), ("U_yy", "U_yy", 1e-10),
                           ("CN", "CN", 1e-9)]:
        assert _rel(mems.field(name), f[key]) <= tol, name
    dxe = mems.field("dksideta").cpu().numpy()
    assert np.abs(dxe - f["Q_dksideta"]).max() <= 1e-12 * np.abs(f["Q_d2ksi"]).max()
    assert _rel(mems.residual(f["u1"]), f["R1"]) <= 1e-9


def test_steps(mems):
    s = load_golden("pma2_steps")
    for i in range(len(s["dt"])):
        dt = mems.step()
        U, Q = mems.state()
        assert abs(dt - s["dt"][i]) <= 1e-17, i
        assert np.abs(U.cpu().numpy() - s["U_new"][i]).max() <= 1e-9, i
        assert _rel(Q, s["Q_val"][i]) <= 1e-12, i
        assert mems.last_stats["nit"] == s["nit"][i], i
    assert abs(mems.time - float(np.sum(s["dt"]))) <= 1e-15


@pytest.mark.parametrize("n", [50, 37])
def test_steps_other_grids_vs_oracle(n):
    """PMA2 steps on grids other than the reference's 51 x 51 against the oracle restatement at
    the same size: an even N takes the PMA solve's even / odd DCT split with no middle entry, an
    odd one a middle entry on another tile layout.  Tolerances as test_steps."""
    import nkhip
    from oracle import pma2_oracle as O
    O.configure(n)
    try:
        unew, qval = O.initial_state()
        m = nkhip.Mems(n=n)
        try:
            m.set_state(unew, qval)
            for i in range(2):
                dt = m.step()
                unew, qval, dto = O.step(unew, qval)
                U, Q = m.state()
                assert abs(dt - dto) <= 1e-17, i
                assert np.abs(U.cpu().numpy() - unew).max() <= 1e-9, i
                assert _rel(Q, qval) <= 1e-12, i
        finally:
            m.close()
    finally:
        O.configure(51)


def test_run_until(mems):
    dts = mems.run(Tf=3.5e-4)
    assert len(dts) == 4 and mems.time >= 3.5e-4


def test_p1_rejected():
    import nkhip
    with pytest.raises(ValueError):
        nkhip.Mems(p=1)
