"""GPU: the droplet stepper (config 3, python_work/droplet.py) against the reference's outputs.

Tolerances (fp64): mesh / old-time fields <= 1e-10 relative (the reference applies the derivative
matrices as COO sparse products, the kernels as stencils: different summation order); the
Newton-Krylov root at f_tol = 1e-7 within 1e-7 absolute (|U| <= ~1); the PMA mesh potential
within 1e-10 relative (the DCT is a dense product here, an FFT in scipy).
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
def drop():
    import nkhip
    z = load_golden("droplet_init")
    d = nkhip.Droplet()
    d.set_state(z["U0"], z["Q0"])
    d.prepare()
    yield d
    d.close()


def test_fields(drop):
    f = load_golden("droplet_fields")
    for name, key, tol in [("d2ksi", "Q_d2ksi", 1e-10), ("d2eta", "Q_d2eta", 1e-10),
                           ("dksideta", "Q_dksideta", 1e-10), ("J", "J", 1e-10),
                           ("Q_dksi", "Q_dksi", 1e-13), ("Q_deta", "Q_deta", 1e-13),
                           ("U_xx", "U_xx", 1e-10), ("U_yy", "U_yy", 1e-10), ("F", "F", 1e-9)]:
        assert _rel(drop.field(name), f[key]) <= tol, name


def test_residual(drop):
    f = load_golden("droplet_fields")
    R = drop.residual(f["u1"], float(f["dt"]))
    assert _rel(R, f["R1"]) <= 1e-11


def test_newton_krylov_fixed_mesh(drop):
    z = load_golden("droplet_nk")
    U = drop.solve(1e-4).cpu().numpy()
    assert np.abs(U - z["U"]).max() <= 1e-7
    assert abs(drop.last_stats["nit"] - int(z["nit"])) <= 1
    assert drop.last_stats["fnorm_inf"] <= 1e-7


@pytest.mark.parametrize("loops", [5, 400])
def test_pma_loop(drop, loops):
    z = load_golden("droplet_pma")
    drop.pma(3e-9, loops)
    Q = drop.field("Q_val")
    assert _rel(Q, z[f"Q_{loops}"]) <= 1e-10


def test_two_full_steps(drop):
    """evolve_with_PDE(1e-4, 3, 1e-2, 3e-9, 400): NK solve + 400 PMA loops per step."""
    z = load_golden("droplet_evolve")
    dts = drop.evolve(2, dt=1e-4, dtmesh=3e-9, pmaloops=400)
    U, Q = drop.state()
    assert np.abs(U.cpu().numpy() - z["U"]).max() <= 1e-6
    assert _rel(Q, z["Q"]) <= 1e-9
    assert dts[0] == 1e-4 and abs(dts[1] - 1.0102881691663517e-4) <= 1e-12


def test_ten_full_steps_every_step(drop):
    """Config 3 over its SURVEY 8(d) length: evolve_with_PDE(1e-4, 11, 1e-2, 3e-9, 400) = S = 10
    steps (droplet.py:360-411), U, Q, dt_n and the Newton count checked after EVERY step against
    the reference's own run (tests/golden/make_golden_droplet.py evolve10).  Bars as for the two
    steps above: U within 1e-6 absolute (NK roots at f_tol = 1e-7, |U| <= ~1), Q within 1e-8
    relative; dt_n carries the exp(-10 |U.new - U.val|) scale recursion (:411), so the roots'
    1e-8-level differences reach it: within 1e-9 absolute (1e-5 relative; the NumPy oracle
    lands 3e-12 from the reference); Newton its +-1."""
    z = load_golden("droplet_evolve10")
    for s in range(10):
        dt = drop.step(1e-4, 3e-9, 400)
        U, Q = drop.state()
        assert np.abs(U.cpu().numpy() - z["U"][s]).max() <= 1e-6, s
        assert _rel(Q, z["Q"][s]) <= 1e-8, s
        assert abs(dt - float(z["dt"][s])) <= 1e-9, (s, dt, float(z["dt"][s]))
        assert abs(drop.last_stats["nit"] - int(z["nit"][s])) <= 1, (s, drop.last_stats)


def test_generic_dropin_on_droplet_residual(drop):
    """The same fixed-mesh solve through nkhip.newton_krylov with the device residual as F."""
    import nkhip
    z = load_golden("droplet_nk")
    U0 = load_golden("droplet_init")["U0"]
    U = nkhip.newton_krylov(lambda u: drop.residual(u, 1e-4), torch.as_tensor(U0, device="cuda"),
                            maxiter=20, f_tol=1e-7)
    assert np.abs(U.cpu().numpy() - z["U"]).max() <= 1e-7


def test_initialise_coalescing_reproduces_reference_init_file(tmp_path):
    """initialise_coalescing_droplets(1000, [[0,0,1,1],[3,0,1,1]], 5e-9, 20) -- 20 000 PMA loops
    from the flat film -- against the reference's own initdrop_coal_1_91-61_... file (its output,
    droplet.py:186-188).  Tolerance: 1e-10 relative (the NumPy oracle lands at 1.4e-12)."""
    import nkhip
    z = load_golden("droplet_init")
    d = nkhip.Droplet()
    try:
        U, Q = d.initialise_coalescing(tofile=str(tmp_path))
        assert _rel(U, z["U0"]) <= 1e-10
        assert _rel(Q, z["Q0"]) <= 1e-12
        U2, Q2 = nkhip.read_init(str(tmp_path / nkhip.droplet.init_filename()))
        assert np.array_equal(U2, U.cpu().numpy()) and np.array_equal(Q2, Q.cpu().numpy())
    finally:
        d.close()



def test_global_memory_fallback(drop, monkeypatch):
    """The droplet kernels' fallback for grids whose planes do not fit LDS (every field in global
    scratch, the PMA loop's plain dense DCT; NKHIP_DROP_GLOBAL=1 forces it, read per launch)
    against the same reference fixtures as the LDS path: the residual and Q after 5 PMA loops."""
    monkeypatch.setenv("NKHIP_DROP_GLOBAL", "1")
    f = load_golden("droplet_fields")
    assert _rel(drop.residual(f["u1"], float(f["dt"])), f["R1"]) <= 1e-11
    drop.pma(3e-9, 5)
    assert _rel(drop.field("Q_val"), load_golden("droplet_pma")["Q_5"]) <= 1e-10
