"""CPU: pin the droplet oracle (NumPy restatement of droplet.py) to the reference's own outputs.

Fixtures: tests/golden/make_golden_droplet.py (the reference module imported with a matplotlib
shim, driven exactly as evolve_with_PDE does).
"""
import os

import numpy as np
import pytest

from conftest import load_golden
from oracle import droplet_oracle as D
from oracle import nk_oracle


def _rel(a, b):
    return float(np.abs(a - b).max() / max(np.abs(b).max(), 1e-300))


@pytest.fixture(scope="module")
def state():
    z = load_golden("droplet_init")
    Q = D.q_ders(z["Q0"])
    F, U = D.step_rhs(z["U0"], Q)
    return z["U0"], z["Q0"], Q, F, U


def test_mesh_and_rhs_fields(state):
    U0, Q0, Q, F, U = state
    f = load_golden("droplet_fields")
    for key, val, tol in [("Q_dksi", Q.dksi, 1e-13), ("Q_deta", Q.deta, 1e-13),
                          ("Q_d2ksi", Q.d2ksi, 1e-10), ("Q_d2eta", Q.d2eta, 1e-10),
                          ("Q_dksideta", Q.dksideta, 1e-10), ("J", Q.J, 1e-10),
                          ("U_xx", U.xx, 1e-10), ("U_yy", U.yy, 1e-10), ("U_dx", U.dx, 1e-10),
                          ("U_dy", U.dy, 1e-10), ("F", F, 1e-9)]:
        assert _rel(val, f[key]) <= tol, key


def test_residual(state):
    U0, Q0, Q, F, U = state
    f = load_golden("droplet_fields")
    R = D.residual(f["u1"], F, float(f["dt"]), U0, Q)
    assert _rel(R, f["R1"]) <= 1e-11


def test_nk_step_fixed_mesh(state):
    U0, Q0, Q, F, U = state
    z = load_golden("droplet_nk")
    u, st = nk_oracle.newton_krylov(lambda u: D.residual(u, F, 1e-4, U0, Q), U0, maxiter=20,
                                    f_tol=1e-7, return_stats=True)
    assert np.abs(u - z["U"]).max() <= 1e-8
    assert st.nit == int(z["nit"]) and st.nfev == int(z["nfev"])


def test_pma_loop(state):
    U0, Q0, Q, F, U = state
    z = load_golden("droplet_pma")
    q5 = D.loop_pma(Q0, U0, 3e-9, 5, Q=Q, U=U)
    assert _rel(q5, z["Q_5"]) <= 1e-13


def test_init_file_roundtrip(tmp_path):
    import nkhip
    z = load_golden("droplet_init")
    p = os.path.join(tmp_path, nkhip.droplet.init_filename())
    nkhip.write_init(p, z["U0"], z["Q0"])
    U, Q = nkhip.read_init(p)
    assert np.array_equal(U, z["U0"]) and np.array_equal(Q, z["Q0"])
    assert os.path.basename(p) == "initdrop_coal_1_91-61_100_0.01_0.01_0.1_0.15.txt"


def test_init_coalescing_reproduces_reference_init_file():
    """The oracle's initialise_coalescing_droplets (droplet.py:132-189, 1000 x 20 PMA loops, about
    a minute on one core) lands on the reference's own initdrop_coal_* output file."""
    z = load_golden("droplet_init")
    u, q = D.init_coalescing()
    assert _rel(u, z["U0"]) <= 1e-11
    assert _rel(q, z["Q0"]) <= 1e-13


def test_evolve_ten_steps_matches_reference():
    """The oracle's evolve_with_PDE over config 3's S = 10 steps (droplet.py:360-411) against the
    reference's own run, every step's dt_n and the final U, Q (tests/golden droplet_evolve10).
    Both sides solve to f_tol = 1e-7 with different summation orders, and dt_n carries the
    exp(-10 |U.new - U.val|) scale recursion (:411): measured 3e-12 (dt), 3e-8 (U), 4e-10 (Q)."""
    z = load_golden("droplet_evolve10")
    u0 = load_golden("droplet_init")
    u, q, _, dts = D.evolve(u0["U0"], u0["Q0"], 10)
    assert np.abs(np.array(dts) - z["dt"]).max() <= 1e-10
    assert np.abs(u - z["U"][-1]).max() <= 1e-6
    assert _rel(q, z["Q"][-1]) <= 1e-8
