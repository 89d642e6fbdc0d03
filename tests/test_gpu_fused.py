"""GPU: the fused Arnoldi step (arnoldi.hip) against the unfused update / JVP / multi-dot path.

The fused launch reads the basis once per Arnoldi step; it changes only the summation order of
the dot products, so both paths must reach the same root (f_tol = 1e-10: agreement to 1e-8 of
the state's scale) with Newton iteration counts within one.  Shapes cover nx not a multiple of
the 60-column wave strip, odd nx, non-square grids and a grid whose band count exceeds its rows.
"""
import os

import numpy as np
import pytest
import torch

from oracle import sh_oracle

pytestmark = pytest.mark.gpu


def _step(ny, nx, fused, ftol=1e-10, seed=2020, steps=1):
    import nkhip
    os.environ["NKHIP_FUSED"] = "1" if fused else "0"
    try:
        m = nkhip.SwiftHohenberg(N=nx, ny=ny, d=0.625 * nx, f_tol=ftol)
        U0 = np.random.default_rng(seed).standard_normal((ny, nx))
        U = torch.as_tensor(U0, device="cuda")
        stats = []
        for _ in range(steps):
            U = m.step(U)
            stats.append(dict(m.last_stats))
        prof = m.kernel_profile()
        m.close()
    finally:
        os.environ.pop("NKHIP_FUSED", None)
    return U0, U.cpu().numpy(), stats, prof


@pytest.mark.parametrize("ny,nx", [(64, 64), (61, 61), (96, 130), (40, 256), (128, 60),
                                   (8, 200), (256, 256), (12, 6)])
def test_fused_matches_unfused(ny, nx):
    U0, a, sa, pa = _step(ny, nx, fused=True)
    _, b, sb, pb = _step(ny, nx, fused=False)
    if nx % 2 == 0:
        assert pa["arnoldi_fused"]["launches"] > 0
    else:  # the fused kernel streams column pairs: odd nx keeps the unfused path
        assert pa["arnoldi_fused"]["launches"] == 0
    assert pb["arnoldi_fused"]["launches"] == 0
    scale = max(1.0, float(np.abs(b).max()))
    assert float(np.abs(a - b).max()) <= 1e-8 * scale
    assert abs(sa[0]["nit"] - sb[0]["nit"]) <= 1
    # the fused path's output is a root of the reference residual (sh_scipy_nk.py:47-49)
    F = sh_oracle.residual(a.reshape(-1), U0.reshape(-1), ny, nx, 0.625, 0.01, 0.2, 1.0)
    assert np.abs(F).max() <= 1e-9


def test_fused_default_tolerance_and_counts():
    """Default f_tol at 512^2 over 3 steps: same roots to the solver tolerance, Krylov work
    within a few percent of the unfused path."""
    _, a, sa, pa = _step(512, 512, fused=True, ftol=None, steps=3)
    _, b, sb, pb = _step(512, 512, fused=False, ftol=None, steps=3)
    scale = max(1.0, float(np.abs(b).max()))
    assert float(np.abs(a - b).max()) <= 1e-5 * scale
    for x, y in zip(sa, sb):
        assert abs(x["nit"] - y["nit"]) <= 1
    na = sum(s["n_arnoldi"] for s in sa)
    nb = sum(s["n_arnoldi"] for s in sb)
    assert abs(na - nb) <= 0.1 * nb + 3
    # most Arnoldi steps run fused (the unfused ones: first step, short-norm fallbacks)
    assert pa["arnoldi_fused"]["launches"] >= 0.5 * na


def test_fused_deterministic():
    _, a, _, _ = _step(96, 130, fused=True)
    _, b, _, _ = _step(96, 130, fused=True)
    assert np.array_equal(a, b)


def _torch_G(y, h, r, k, g):
    """G(y) = y/k - (L y + g y^2 - y^3)/2 with L = -Lap^2 - 2 Lap + (r-1) I by periodic rolls
    (sh_scipy_nk.py:32-39,49), an fp64 torch reference independent of the HIP stencils."""
    e = 1.0 / h ** 2

    def lap(a):
        return e * (torch.roll(a, 1, 0) + torch.roll(a, -1, 0) + torch.roll(a, 1, 1)
                    + torch.roll(a, -1, 1) - 4 * a)

    la = lap(y)
    Ly = -lap(la) - 2 * la + (r - 1) * y
    return y / k - (Ly + g * y * y - y * y * y) / 2


@pytest.mark.parametrize("ny,nx", [(64, 64), (40, 130), (96, 62), (16, 4)])
@pytest.mark.parametrize("nv", [1, 5, 18, 35])
@pytest.mark.parametrize("ext", [False, True])
def test_fused_kernel_vs_torch(ny, nx, nv, ext):
    _check_fused_vs_torch(ny, nx, nv, ext)


@pytest.mark.parametrize("ny,nx", [(40, 130), (24, 600)])
@pytest.mark.parametrize("nv", list(range(1, 36)))
@pytest.mark.parametrize("ext", [False, True])
def test_fused_kernel_every_basis_length(ny, nx, nv, ext):
    """Every instantiation of the fused kernel (each basis length has its own, in both layouts'
    ranges, with and without z) against the torch reference, on short bands (the alternating
    march) and ragged widths.  A round-6 build that passed the solver tests computed w' wrong at
    wave boundaries in the nv-7 wide kernel with z only (the compiler's output for that one
    instantiation, profiles/r06_short_slab.md section 8): no instantiation is trusted untested."""
    _check_fused_vs_torch(ny, nx, nv, ext)


def _check_fused_vs_torch(ny, nx, nv, ext):
    import nkhip
    gen = torch.Generator(device="cpu").manual_seed(nv * 100 + nx)
    rnd = lambda: torch.randn(ny, nx, generator=gen, dtype=torch.float64).cuda()  # noqa: E731
    V = [rnd() for _ in range(nv)]
    coef = [float(c) for c in torch.randn(nv, generator=gen, dtype=torch.float64)]
    w, x0 = rnd(), rnd()
    z = rnd() if ext else None
    h, r, k, g, tau = 0.625, 0.01, 0.2, 1.0, 0.75
    G0 = _torch_G(x0, h, r, k, g)
    zs, sc = 0.5, 1e-3
    v, wo, dots = nkhip.sh_arnoldi_fused(V, coef, w, tau, x0, G0, h, r, k, g, zs, sc, z=z)
    vr = tau * w
    for c, Vi in zip(coef, V):
        vr = vr + c * Vi
    zr = z if ext else vr
    wr = (_torch_G(x0 + sc * zs * zr, h, r, k, g) - G0) / sc
    assert float((v - vr).abs().max()) <= 1e-13 * float(vr.abs().max())
    assert float((wo - wr).abs().max()) <= 1e-9 * float(wr.abs().max())
    ref = [float((wr * Vi).sum()) for Vi in V] + [float((wr * vr).sum())]
    ref += [float((vr * Vi).sum()) for Vi in V] + [float((vr * vr).sum()), float((wr * wr).sum())]
    scale_w = float(wr.norm()) * float(max(Vi.norm() for Vi in V + [vr]))
    scale_v = float(vr.norm()) * float(max(Vi.norm() for Vi in V + [vr]))
    for i, (a, b) in enumerate(zip(dots, ref)):
        scale = scale_w if (i <= nv or i == 2 * nv + 2) else scale_v
        assert abs(a - b) <= 1e-10 * scale, (i, a, b)


@pytest.mark.parametrize("devctl", ["1", "0"])
@pytest.mark.parametrize("overlap", ["0", "1"])
@pytest.mark.parametrize("nranks,ny_total,nx", [(2, 64, 64), (3, 96, 130), (4, 48, 40),
                                                  (8, 1024, 1024)])
def test_fused_slabs_match_single_slab(nranks, ny_total, nx, overlap, devctl, monkeypatch):
    """Row slabs through the fused kernel: every rank evaluates y on its edge rows, the loopback
    communicator exchanges them (the RCCL path's protocol), and the fused pass takes them as its
    halo rows.  Same root as the single periodic slab, and the fused kernel did run on each slab.
    devctl "1" (the default with a communicator): the Arnoldi control runs on the device, every
    rank's control kernel taking the same decisions from the same all-reduced results."""
    import nkhip
    from conftest import load_golden, run_slabs
    # "1": interior rows on a side stream during the edge exchange, edge bands after it
    monkeypatch.setenv("NKHIP_SLAB_OVERLAP", overlap)
    monkeypatch.setenv("NKHIP_DEVCTL", devctl)
    U0 = np.random.default_rng(7).standard_normal((ny_total, nx))
    single = nkhip.SwiftHohenberg(N=nx, ny=ny_total, d=0.625 * nx, f_tol=1e-10)
    ref = single.step(torch.as_tensor(U0, device="cuda")).cpu().numpy()
    ref_nit = single.last_stats["nit"]
    single.close()
    comms = nkhip.loopback_comms(nranks)
    out, profs, nits, devs = [None] * nranks, [None] * nranks, [None] * nranks, [None] * nranks

    def run(p):
        stream = torch.cuda.Stream()
        with torch.cuda.stream(stream):
            row0, ny = nkhip.slab_rows(ny_total, p, nranks)
            m = nkhip.SwiftHohenberg(N=nx, ny=ny_total, d=0.625 * nx, f_tol=1e-10,
                                     comm=comms[p], ny_local=ny, stream=stream)
            u = torch.as_tensor(U0[row0:row0 + ny].copy(), device="cuda")
            out[p] = m.step(u).cpu().numpy()
            nits[p] = m.last_stats["nit"]
            devs[p] = m.last_stats["n_device_steps"]
            profs[p] = m.kernel_profile()
            stream.synchronize()
            m.close()

    run_slabs(comms, run)
    for pr in profs:
        assert pr["arnoldi_fused"]["launches"] > 0
        assert pr["arnoldi_edge"]["launches"] == pr["arnoldi_fused"]["launches"]
        if overlap == "1" and ny_total // nranks >= 12:
            assert pr["arnoldi_slab_edges"]["launches"] == pr["arnoldi_fused"]["launches"]
    assert len(set(nits)) == 1 and abs(nits[0] - ref_nit) <= 1
    assert len(set(devs)) == 1 and ((devs[0] > 0) == (devctl == "1")), devs
    got = np.concatenate(out, axis=0)
    assert np.abs(got - ref).max() <= 1e-8 * max(1.0, np.abs(ref).max())
    F = sh_oracle.residual(got.reshape(-1), U0.reshape(-1), ny_total, nx, 0.625, 0.01, 0.2, 1.0)
    assert np.abs(F).max() <= 1e-9


@pytest.mark.parametrize("ny,nx", [(64, 64), (40, 130), (24, 600), (16, 4), (8, 512)])
@pytest.mark.parametrize("ext", [False, True])
def test_fused_kernel_edges_identical(ny, nx, ext):
    """Block halos read from the entries' edge arrays (nk_sh_arnoldi_fused_edges) are the same
    values as read from the vectors: v, w' and every dot product are bitwise equal, and the edge
    arrays the kernel writes for v and w' equal nk_edge_gather of the outputs."""
    import nkhip
    nv = 7
    gen = torch.Generator(device="cpu").manual_seed(nx + ny)
    rnd = lambda: torch.randn(ny, nx, generator=gen, dtype=torch.float64).cuda()  # noqa: E731
    V = [rnd() for _ in range(nv)]
    coef = [float(c) for c in torch.randn(nv, generator=gen, dtype=torch.float64)]
    w, x0 = rnd(), rnd()
    z = rnd() if ext else None
    args = (V, coef, w, 0.75, x0, None, 0.625, 0.01, 0.2, 1.0, 0.5, 1e-3)
    v1, w1, d1 = nkhip.sh_arnoldi_fused(*args, z=z)
    E = [nkhip.edge_gather(t) for t in V + [w]]
    Ev = torch.full_like(E[0], float("nan"))
    Ew = torch.full_like(E[0], float("nan"))
    v2, w2, d2 = nkhip.sh_arnoldi_fused(*args, z=z, E=E, Ev_out=Ev, Ew_out=Ew)
    assert torch.equal(v1, v2) and torch.equal(w1, w2) and d1 == d2
    assert torch.equal(Ev, nkhip.edge_gather(v2))
    assert torch.equal(Ew, nkhip.edge_gather(w2))


@pytest.mark.parametrize("ny,nx", [(64, 600), (128, 512)])
def test_edges_identical_solve(ny, nx, monkeypatch):
    """The solver with edge arrays (default: the fused kernel's block halos, the FD-JVP's block
    side columns) and without (NKHIP_EDGES=0) is bitwise the same."""
    monkeypatch.setenv("NKHIP_EDGES", "0")
    _, a, sa, pa = _step(ny, nx, fused=True)
    monkeypatch.delenv("NKHIP_EDGES")
    _, b, sb, pb = _step(ny, nx, fused=True)
    assert np.array_equal(a, b) and sa == sb
    assert pb["arnoldi_fused"]["launches"] > 0


@pytest.mark.parametrize("ny,nx", [(64, 600), (128, 512)])
def test_combo_edges_identical_solve(ny, nx, monkeypatch):
    """The LGMRES combinations write their outputs' edge arrays themselves (EdgeOut): the same
    solve, bitwise, as with an edge_gather pass after each (NKHIP_COMBO_EDGES=0), and no
    edge_gather launch is left.  nx = 600 puts the last group border at the row end."""
    monkeypatch.setenv("NKHIP_COMBO_EDGES", "0")
    _, a, sa, pa = _step(ny, nx, fused=True)
    monkeypatch.delenv("NKHIP_COMBO_EDGES")
    _, b, sb, pb = _step(ny, nx, fused=True)
    assert np.array_equal(a, b) and sa == sb
    assert pa.get("edge_gather", {}).get("launches", 0) > 0
    assert pb.get("edge_gather", {}).get("launches", 0) == 0


@pytest.mark.parametrize("ny,nx,fused", [(64, 64, True), (61, 61, False), (256, 256, True),
                                         (128, 600, True), (96, 130, False)])
def test_speculative_jvp_identical(ny, nx, fused, monkeypatch):
    """The line search's speculative first JVP of the next LGMRES call (NewtonKrylov::line_search:
    queued behind the s = 1 trial, run by the device only if that trial passes the Armijo test and
    the iteration goes on, with the host's FD step from the same reduction values) leaves the
    solve bitwise as without it (NKHIP_SPEC_JVP=0): same roots, same Newton / F-eval / JVP
    counts, and the same FD-JVP launch count (a pass the trial cancelled leaves the profile)."""
    monkeypatch.setenv("NKHIP_SPEC_JVP", "0")
    _, a, sa, pa = _step(ny, nx, fused=fused, steps=2)
    monkeypatch.delenv("NKHIP_SPEC_JVP")
    _, b, sb, pb = _step(ny, nx, fused=fused, steps=2)
    assert np.array_equal(a, b) and sa == sb
    assert sum(s["nit"] for s in sb) > 2  # line searches that armed it
    assert pa["sh_fdjvp"]["launches"] == pb["sh_fdjvp"]["launches"]


def test_speculative_jvp_backtracking(monkeypatch):
    """The same on the reference's backtracking step (nk_n61_amp3_backtrack: 5 of 13 Newton
    iterations backtrack, so the speculative pass is cancelled there and runs elsewhere)."""
    import nkhip
    from conftest import load_golden
    z = load_golden("nk_n61_amp3_backtrack")
    N = int(z["N"])
    out = {}
    for mode in ("0", "1"):
        monkeypatch.setenv("NKHIP_SPEC_JVP", mode)
        m = nkhip.SwiftHohenberg(N=N, d=float(z["d"]), k=float(z["k"]), r=float(z["r"]),
                                 g=float(z["g"]), f_tol=None if np.isnan(z["f_tol"])
                                 else float(z["f_tol"]))
        U = m.step(torch.as_tensor(z["traj"][0].reshape(N, N), device="cuda"))
        out[mode] = (U.cpu().numpy(), dict(m.last_stats), list(m.step_log()),
                     m.kernel_profile()["sh_fdjvp"]["launches"])
        m.close()
    assert np.array_equal(out["0"][0], out["1"][0])
    assert out["0"][1:] == out["1"][1:]
    assert sum(s < 1 for s in out["1"][2]) >= 1


@pytest.mark.parametrize("ny,nx", [(64, 64), (128, 60), (96, 130), (256, 256), (40, 512),
                                   (1024, 1024)])
@pytest.mark.parametrize("tail", ["0", "1"])
def test_device_control_matches_host(ny, nx, tail, monkeypatch):
    """Device-side Arnoldi control (arnctl.hip: the Givens update, residual test, Gram row and
    MGS coefficients computed by a one-wave kernel between the fused launches, handed back to the
    host loop at the stop): the same root as the host loop to 1e-8 of the state's scale, Newton
    counts within one, a root of the oracle residual, and the device did run steps."""
    monkeypatch.setenv("NKHIP_DEVCTL", "0")
    U0, a, sa, _ = _step(ny, nx, fused=True, steps=2)
    monkeypatch.setenv("NKHIP_DEVCTL", "1")
    monkeypatch.setenv("NKHIP_ARN_TAIL", tail)  # 1: reduction + control in the fused launch's tail
    _, b, sb, pb = _step(ny, nx, fused=True, steps=2)
    assert all(s["n_device_steps"] == 0 for s in sa)
    assert sum(s["n_device_steps"] for s in sb) > 0
    assert pb["arnoldi_ctl"]["launches"] > 0
    for x, y in zip(sa, sb):
        assert abs(x["nit"] - y["nit"]) <= 1 and y["status"] == 0
        # the device steps are a subset of the Arnoldi steps
        assert y["n_device_steps"] < y["n_arnoldi"]
    assert np.abs(a - b).max() <= 1e-8 * max(1.0, np.abs(a).max())


def test_device_control_default_tolerance():
    """At scipy's default f_tol the device-controlled solve reaches a root of the oracle
    residual with the host loop's Newton count (within one), over several time steps."""
    ny = nx = 128
    os.environ["NKHIP_DEVCTL"] = "1"
    try:
        U0, b, sb, _ = _step(ny, nx, fused=True, ftol=None, steps=1)
    finally:
        os.environ.pop("NKHIP_DEVCTL", None)
    _, a, sa, _ = _step(ny, nx, fused=True, ftol=None, steps=1)
    assert abs(sa[0]["nit"] - sb[0]["nit"]) <= 1 and sb[0]["n_device_steps"] > 0
    F = sh_oracle.residual(b.reshape(-1), U0.reshape(-1), ny, nx, 0.625, 0.01, 0.2, 1.0)
    assert np.abs(F).max() <= 1.01 * np.finfo(float).eps ** (1 / 3)


def _mbox_expected(nv, nx):
    """Whether the fused kernel's grid takes the mailbox: the vector-pair layout (nv >= 19;
    the wide layout keeps its packed halo loads) with nx a multiple of its mailbox instantiation's
    128-column blocks and two blocks per band at least."""
    return nv >= 19 and nx % 128 == 0 and nx // 128 >= 2


@pytest.mark.parametrize("ny,nx", [(64, 1024), (40, 512), (24, 2048), (32, 384)])
@pytest.mark.parametrize("nv", [1, 6, 18, 19, 27, 35])
def test_fused_kernel_mailbox(ny, nx, nv, monkeypatch):
    """Block halos through the mailbox (arnoldi.hip "Mailbox": the blocks of a band publish u on
    their edge columns): bitwise the same v, w' and dots as every consumer recomputing its halo
    pair itself (NKHIP_ARN_MBOX=2, the path a missing neighbour takes); v bitwise and w', dots
    within rounding of the packed halo loads (NKHIP_ARN_MBOX=0, which sum the halo in another
    order); the mailbox ran exactly where the grid allows it."""
    import nkhip
    gen = torch.Generator(device="cpu").manual_seed(nv * 7 + nx + ny)
    rnd = lambda: torch.randn(ny, nx, generator=gen, dtype=torch.float64).cuda()  # noqa: E731
    V = [rnd() for _ in range(nv)]
    coef = [float(c) for c in torch.randn(nv, generator=gen, dtype=torch.float64)]
    w, x0 = rnd(), rnd()
    args = (V, coef, w, 0.75, x0, None, 0.625, 0.01, 0.2, 1.0, 0.5, 1e-3)
    res, used = {}, {}
    for mode in ("1", "2", "0"):
        monkeypatch.setenv("NKHIP_ARN_MBOX", mode)
        n0 = nkhip.arnoldi_mbox_launches()
        res[mode] = nkhip.sh_arnoldi_fused(*args)
        used[mode] = nkhip.arnoldi_mbox_launches() - n0
    on = _mbox_expected(nv, nx)
    assert used == {"1": int(on), "2": int(on), "0": 0}, used
    (v1, w1, d1), (v2, w2, d2), (v0, w0, d0) = res["1"], res["2"], res["0"]
    assert torch.equal(v1, v2) and torch.equal(w1, w2) and d1 == d2
    assert torch.equal(v1, v0)
    assert float((w1 - w0).abs().max()) <= 1e-12 * float(w0.abs().max())
    scale = float(w0.norm()) * float(max(t.norm() for t in V + [v0])) + float(v0.norm()) ** 2
    assert max(abs(a - b) for a, b in zip(d1, d0)) <= 1e-12 * scale


@pytest.mark.parametrize("ny,nx", [(128, 1024), (64, 512)])
def test_mailbox_solve(ny, nx, monkeypatch):
    """The solver with the mailbox (default) is bitwise the solver whose consumers all recompute
    their halo pairs (NKHIP_ARN_MBOX=2), and reaches the root of the packed-halo solver
    (NKHIP_ARN_MBOX=0) to 1e-8 of the state's scale; the mailbox ran."""
    import nkhip
    n0 = nkhip.arnoldi_mbox_launches()
    U0, a, sa, pa = _step(ny, nx, fused=True)
    assert nkhip.arnoldi_mbox_launches() - n0 >= 1  # the vector-pair layout's (nv >= 19)
    monkeypatch.setenv("NKHIP_ARN_MBOX", "2")
    _, b, sb, _ = _step(ny, nx, fused=True)
    monkeypatch.setenv("NKHIP_ARN_MBOX", "0")
    n1 = nkhip.arnoldi_mbox_launches()
    _, c, sc_, _ = _step(ny, nx, fused=True)
    assert nkhip.arnoldi_mbox_launches() == n1
    assert np.array_equal(a, b) and sa == sb
    assert np.abs(a - c).max() <= 1e-8 * max(1.0, np.abs(c).max())
    assert abs(sa[0]["nit"] - sc_[0]["nit"]) <= 1
    F = sh_oracle.residual(a.reshape(-1), U0.reshape(-1), ny, nx, 0.625, 0.01, 0.2, 1.0)
    assert np.abs(F).max() <= 1e-9


def test_fused_kernel_mailbox_every_length(monkeypatch):
    """Every basis length 1..35 (one kernel instantiation each; the mailbox from 19 on) at 32x1024:
    bitwise the recompute path's v, w' and dots, and v, w' within rounding of an fp64 torch
    reference (sh_scipy_nk.py:47-49 residual, _nonlin.py:1505-1513 quotient)."""
    import nkhip
    ny, nx = 32, 1024
    h, r, k, g, tau, zs, sc = 0.625, 0.01, 0.2, 1.0, 0.75, 0.5, 1e-3
    gen = torch.Generator(device="cpu").manual_seed(11)
    rnd = lambda: torch.randn(ny, nx, generator=gen, dtype=torch.float64).cuda()  # noqa: E731
    Vall = [rnd() for _ in range(35)]
    w, x0 = rnd(), rnd()
    G0 = _torch_G(x0, h, r, k, g)
    for nv in range(1, 36):
        print("nv", nv, flush=True)
        V = Vall[:nv]
        coef = [0.3 / nv * (1 + (i % 3)) for i in range(nv)]
        n0 = nkhip.arnoldi_mbox_launches()
        monkeypatch.setenv("NKHIP_ARN_MBOX", "1")
        v1, w1, d1 = nkhip.sh_arnoldi_fused(V, coef, w, tau, x0, G0, h, r, k, g, zs, sc)
        monkeypatch.setenv("NKHIP_ARN_MBOX", "2")
        v2, w2, d2 = nkhip.sh_arnoldi_fused(V, coef, w, tau, x0, G0, h, r, k, g, zs, sc)
        assert nkhip.arnoldi_mbox_launches() - n0 == (2 if nv >= 19 else 0), nv
        assert torch.equal(v1, v2) and torch.equal(w1, w2) and d1 == d2, nv
        vr = tau * w
        for c, Vi in zip(coef, V):
            vr = vr + c * Vi
        wr = (_torch_G(x0 + sc * zs * vr, h, r, k, g) - G0) / sc
        assert float((v1 - vr).abs().max()) <= 1e-13 * float(vr.abs().max()), nv
        assert float((w1 - wr).abs().max()) <= 1e-9 * float(wr.abs().max()), nv


@pytest.mark.parametrize("ny,nx", [(512, 4096), (64, 1024), (40, 130), (24, 600), (8, 512)])
@pytest.mark.parametrize("nv", [1, 4, 8, 18, 19, 27, 35])
@pytest.mark.parametrize("ext", [False, True])
def test_fused_kernel_march_direction(ny, nx, nv, ext, monkeypatch):
    """Alternating march (arnoldi.hip "March direction": odd bands march up their rows so that
    adjacent bands read their shared halo rows at the same time) against every band marching
    down (NKHIP_ARN_ALT=0, the kernel before round 6): v, w' and the edge arrays written for them
    bitwise the same -- the stencil adds the rows either side of the centre commutatively -- and
    the dot products, whose per-wave row order is reversed in the odd bands, within rounding.
    512 x 4096 is the N = 8 rank's slab of the 4096^2 headline."""
    import nkhip
    gen = torch.Generator(device="cpu").manual_seed(nv * 13 + nx + ny + int(ext))
    rnd = lambda: torch.randn(ny, nx, generator=gen, dtype=torch.float64).cuda()  # noqa: E731
    V = [rnd() for _ in range(nv)]
    coef = [float(c) for c in torch.randn(nv, generator=gen, dtype=torch.float64)]
    w, x0 = rnd(), rnd()
    z = rnd() if ext else None
    args = (V, coef, w, 0.75, x0, None, 0.625, 0.01, 0.2, 1.0, 0.5, 1e-3)
    E = [nkhip.edge_gather(t) for t in V + [w]]
    res = {}
    for alt in ("0", "1"):
        monkeypatch.setenv("NKHIP_ARN_ALT", alt)
        Ev = torch.full_like(E[0], float("nan"))
        Ew = torch.full_like(E[0], float("nan"))
        v, wo, d = nkhip.sh_arnoldi_fused(*args, z=z, E=E, Ev_out=Ev, Ew_out=Ew)
        res[alt] = (v, wo, d, Ev, Ew)
    (v0, w0, d0, Ev0, Ew0), (v1, w1, d1, Ev1, Ew1) = res["0"], res["1"]
    assert torch.equal(v0, v1) and torch.equal(w0, w1)
    assert torch.equal(Ev0, Ev1) and torch.equal(Ew0, Ew1)
    scale = float(w0.norm()) * float(max(t.norm() for t in V + [v0])) + float(v0.norm()) ** 2
    assert max(abs(a - b) for a, b in zip(d0, d1)) <= 1e-13 * scale


@pytest.mark.parametrize("ny,nx", [(512, 1024), (96, 130)])
def test_march_direction_solve(ny, nx, monkeypatch):
    """The solver with the alternating march (default) reaches the root of the all-down march
    (NKHIP_ARN_ALT=0) to 1e-8 of the state's scale with Newton counts within one, is
    deterministic, and its output is a root of the reference residual (sh_scipy_nk.py:47-49)."""
    monkeypatch.setenv("NKHIP_ARN_ALT", "0")
    U0, a, sa, _ = _step(ny, nx, fused=True)
    monkeypatch.setenv("NKHIP_ARN_ALT", "1")
    _, b, sb, pb = _step(ny, nx, fused=True)
    _, c, sc_, _ = _step(ny, nx, fused=True)
    assert np.array_equal(b, c) and sb == sc_
    assert pb["arnoldi_fused"]["launches"] > 0
    assert abs(sa[0]["nit"] - sb[0]["nit"]) <= 1
    assert np.abs(a - b).max() <= 1e-8 * max(1.0, np.abs(a).max())
    F = sh_oracle.residual(b.reshape(-1), U0.reshape(-1), ny, nx, 0.625, 0.01, 0.2, 1.0)
    assert np.abs(F).max() <= 1e-9


@pytest.mark.parametrize("ny,nx,nv,alt", [(512, 4096, 24, "1"), (512, 4096, 8, "1"),
                                          (4096, 4096, 8, "0"), (4096, 4096, 24, "0")])
def test_march_direction_auto(ny, nx, nv, alt, monkeypatch):
    """Without NKHIP_ARN_ALT the host takes the alternating march for bands of at most 32 rows
    (arnoldi.hip arnoldi_alt_mode): the N = 8 rank's 512-row slab (pair layout: 32-row bands,
    wide: 16) runs it, the 4096-row grid (64- and 256-row bands) does not.  The dot products of
    the two marches differ in rounding, so bitwise equality of every output names the path."""
    import nkhip
    gen = torch.Generator(device="cpu").manual_seed(nv + ny)
    rnd = lambda: torch.randn(ny, nx, generator=gen, dtype=torch.float64).cuda()  # noqa: E731
    V = [rnd() for _ in range(nv)]
    coef = [float(c) for c in torch.randn(nv, generator=gen, dtype=torch.float64)]
    w, x0 = rnd(), rnd()
    args = (V, coef, w, 0.75, x0, None, 0.625, 0.01, 0.2, 1.0, 0.5, 1e-3)
    monkeypatch.delenv("NKHIP_ARN_ALT", raising=False)
    v, wo, d = nkhip.sh_arnoldi_fused(*args)
    monkeypatch.setenv("NKHIP_ARN_ALT", alt)
    v1, w1, d1 = nkhip.sh_arnoldi_fused(*args)
    monkeypatch.setenv("NKHIP_ARN_ALT", "1" if alt == "0" else "0")
    v2, w2, d2 = nkhip.sh_arnoldi_fused(*args)
    assert torch.equal(v, v1) and torch.equal(wo, w1) and d == d1
    assert torch.equal(v, v2) and torch.equal(wo, w2) and d != d2  # the other march: dots only
