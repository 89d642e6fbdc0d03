"""GPU: the HIP stencil and BLAS-1 kernels against the reference's golden vectors and the oracle.

Tolerance (fp64): operator outputs within 1e-13 relative (max-norm) of the reference's CSR SpMV;
the stencil sums in a different order than CSR, so bitwise equality is not expected.
"""
import numpy as np
import pytest
import torch

from conftest import load_golden
from oracle import sh_oracle

pytestmark = pytest.mark.gpu

OPS = ["ops_n5_d2", "ops_n61", "ops_n64", "ops_n128_h0625"]


def _t(a):
    return torch.as_tensor(np.ascontiguousarray(a), dtype=torch.float64, device="cuda")


def _rel(a, b):
    a = a.detach().cpu().numpy() if isinstance(a, torch.Tensor) else a
    return float(np.abs(a - b).max() / max(np.abs(b).max(), 1e-300))


@pytest.mark.parametrize("name", OPS)
def test_lap5_and_sh13_vs_reference(name):
    import nkhip
    z = load_golden(name)
    N, h, r = int(z["N"]), float(z["h"]), float(z["r"])
    v = _t(z["v"])
    assert _rel(nkhip.lap5_apply(v, 1.0 / h ** 2, N, N), z["lap_v"]) <= 1e-13
    assert _rel(nkhip.sh13_apply(v, h, r, N, N), z["L_v"]) <= 1e-13


@pytest.mark.parametrize("ny,nx", [(1, 1), (1, 6), (2, 2), (3, 5), (4, 4), (5, 7), (7, 2),
                                   (9, 256), (33, 258), (64, 512), (130, 1030), (256, 96)])
def test_stencils_odd_even_rect_tiny(ny, nx):
    import nkhip
    rng = np.random.default_rng(ny * 1000 + nx)
    v = rng.standard_normal(ny * nx)
    h, r = 0.625, 0.01
    y = nkhip.sh13_apply(_t(v), h, r, ny, nx)
    assert _rel(y, sh_oracle.sh13(v, ny, nx, h, r)) <= 1e-13
    y5 = nkhip.lap5_apply(_t(v), 1 / h ** 2, ny, nx)
    assert _rel(y5, sh_oracle.lap5(v, ny, nx, 1 / h ** 2)) <= 1e-13


def test_residual_vs_reference():
    import nkhip
    z = load_golden("residual_n61")
    F = nkhip.sh_residual(_t(z["u"]), _t(z["uo"]), float(z["h"]), float(z["r"]), float(z["k"]),
                          float(z["g"]), 61, 61)
    assert _rel(F, z["F"]) <= 1e-12


@pytest.mark.parametrize("N", [61, 64, 256])
def test_residual_and_jvp_vs_oracle(N):
    import nkhip
    rng = np.random.default_rng(N)
    u, uo, v = (rng.standard_normal(N * N) for _ in range(3))
    h, r, k, g = 0.625, 0.01, 0.2, 1.0
    F = nkhip.sh_residual(_t(u), _t(uo), h, r, k, g, N, N)
    assert _rel(F, sh_oracle.residual(u, uo, N, N, h, r, k, g)) <= 1e-12
    J = nkhip.sh_jvp(_t(u), _t(v), h, r, k, g, N, N)
    assert _rel(J, sh_oracle.jvp(u, v, N, N, h, r, k, g)) <= 1e-12


@pytest.mark.parametrize("N", [61, 64, 256])
def test_fd_matvec_vs_oracle(N):
    """nk_sh_fdjvp = KrylovJacobian.matvec's (F(x0 + sc v) - F(x0))/sc (_nonlin.py:1505-1509) on the
    x-dependent part G of the residual.  A difference quotient amplifies the rounding of G by 1/sc
    (with scipy's own step, omega = sqrt(eps)|x0|/|F0| ~ 1e-10 here, that noise is ~1e-4 of the
    result), so the kernel arithmetic is checked at a step where the noise is ~1e-9: against the
    oracle's quotient to 1e-7 relative, and against the analytic J v to the O(sc) truncation."""
    import nkhip
    rng = np.random.default_rng(N + 1)
    x0, z = rng.standard_normal(N * N), rng.standard_normal(N * N)
    h, r, k, g = 0.625, 0.01, 0.2, 1.0

    def G(w):
        return w / k - (sh_oracle.sh13(w, N, N, h, r) + g * w * w - w * w * w) / 2

    G0 = G(x0)
    zs = 1.0 / np.linalg.norm(z)
    sc = 1e-4
    y = nkhip.sh_fdjvp(_t(x0), _t(G0), _t(z), h, r, k, g, zs, sc, N, N)
    ref = (G(x0 + sc * zs * z) - G0) / sc
    assert _rel(y, ref) <= 1e-7
    # and it is the Jacobian product up to the FD truncation error O(sc)
    assert _rel(y, sh_oracle.jvp(x0, zs * z, N, N, h, r, k, g)) <= 1e-5


@pytest.mark.parametrize("n", [1, 7, 2047, 2048, 2049, 100_001, 1 << 20])
def test_blas1_vs_torch(n):
    import nkhip
    g = torch.Generator(device="cpu").manual_seed(n)
    x = torch.randn(n, dtype=torch.float64, generator=g).cuda()
    y = torch.randn(n, dtype=torch.float64, generator=g).cuda()
    assert abs(nkhip.dot(x, y) - float(x @ y)) <= 1e-12 * float(x.abs() @ y.abs())
    assert abs(nkhip.nrm2(x) - float(x.norm())) <= 1e-13 * float(x.norm())
    assert nkhip.maxnorm(x) == float(x.abs().max())
    V = [torch.randn(n, dtype=torch.float64, generator=g).cuda() for _ in range(5)]
    d = nkhip.mdot(V, x)
    for vi, di in zip(V, d):
        assert abs(di - float(vi @ x)) <= 1e-12 * float(vi.abs() @ x.abs())
    y2 = y.clone()
    nkhip.maxpy(V, [0.5, -1.0, 2.0, 0.0, 3.0], y2)
    ref = y + 0.5 * V[0] - V[1] + 2 * V[2] + 3 * V[4]
    assert float((y2 - ref).abs().max()) <= 1e-13 * float(ref.abs().max())
    y3 = y.clone()
    nkhip.axpy(2.5, x, y3)
    assert float((y3 - (y + 2.5 * x)).abs().max()) <= 1e-14 * float((y + 2.5 * x).abs().max())
    nkhip.scal(-3.0, y3)


def test_blas1_unaligned_views():
    import nkhip
    x = torch.randn(1001, dtype=torch.float64, device="cuda")
    y = torch.randn(1001, dtype=torch.float64, device="cuda")
    a, b = x[1:], y[1:]  # 8-byte offset: the scalar (non-double2) kernels run
    assert abs(nkhip.dot(a, b) - float(a @ b)) <= 1e-12 * float(a.abs() @ b.abs())
    assert nkhip.maxnorm(a) == float(a.abs().max())


def test_maxnorm_propagates_nan():
    import nkhip
    x = torch.randn(5000, dtype=torch.float64, device="cuda")
    x[1234] = float("nan")
    assert np.isnan(nkhip.maxnorm(x))


def test_reductions_are_deterministic():
    import nkhip
    x = torch.randn(3_000_001, dtype=torch.float64, device="cuda")
    y = torch.randn(3_000_001, dtype=torch.float64, device="cuda")
    vals = {nkhip.dot(x, y) for _ in range(5)}
    assert len(vals) == 1


def test_rejects_wrong_dtype_and_host_tensors():
    import nkhip
    with pytest.raises(TypeError):
        nkhip.sh13_apply(torch.zeros(16, 16, device="cuda", dtype=torch.float32), 0.6, 0.01)
    with pytest.raises(TypeError):
        nkhip.sh13_apply(torch.zeros(16, 16, dtype=torch.float64), 0.6, 0.01)


def test_march_and_point_kernels_agree_bitwise():
    """Even nx runs the marching kernel (bands alternate direction), odd nx the point kernel; the
    symmetric pairing of the stencil sums makes both produce identical bits on a shared grid."""
    import nkhip
    rng = np.random.default_rng(5)
    v = rng.standard_normal((64, 66))
    h, r = 0.625, 0.01
    y_march = nkhip.sh13_apply(_t(v), h, r).cpu().numpy()
    # same values through the point kernel: an 8-byte-offset (unaligned) view forces it
    buf = torch.zeros(64 * 66 + 1, dtype=torch.float64, device="cuda")
    buf[1:] = _t(v.reshape(-1))
    out = torch.zeros(64 * 66 + 1, dtype=torch.float64, device="cuda")
    nkhip.sh13_apply(buf[1:], h, r, 64, 66, out=out[1:])
    assert np.array_equal(y_march.reshape(-1), out[1:].cpu().numpy())


@pytest.mark.parametrize("op", ["lap5", "sh13"])
def test_config2_1024(op):
    """BASELINE config 2: the 1024^2 fp64 periodic Laplacian (and the 13-point L) on the grid
    and input the bench measures (v = default_rng(7).standard_normal, h = 0.625) vs the oracle
    stencils, themselves pinned to the reference's CSR matrices (test_oracle.py)."""
    import nkhip
    n, h, r = 1024, 0.625, 0.01
    v_np = np.random.default_rng(7).standard_normal(n * n)
    v = torch.as_tensor(v_np.reshape(n, n), device="cuda")
    if op == "lap5":
        y = nkhip.lap5_apply(v, 1 / h ** 2).cpu().numpy().reshape(-1)
        ref = sh_oracle.lap5(v_np, n, n, 1 / h ** 2)
    else:
        y = nkhip.sh13_apply(v, h, r).cpu().numpy().reshape(-1)
        ref = sh_oracle.sh13(v_np, n, n, h, r)
    assert np.abs(y - ref).max() <= 1e-13 * max(1.0, np.abs(ref).max())


@pytest.mark.parametrize("op", ["lap5", "sh13"])
@pytest.mark.parametrize("ny,nx", [(2048, 1024), (2056, 1024), (6, 8), (3, 10), (7, 700), (5, 258)])
def test_tile_and_march_operators(op, ny, nx):
    """The pure operators take the one-row-per-thread tile kernel up to 2^21 points (config 2's
    1024^2) and the march kernel above: both against the oracle stencils on either side of the
    switch (2048 x 1024 = 2^21: tile; 2056 x 1024: march), on the smallest grids and on rows that
    end inside a wave (700, 258 columns: the lane exchange's row-end lanes load their own)."""
    import nkhip
    h, r = 0.625, 0.01
    v_np = np.random.default_rng(ny + nx).standard_normal(ny * nx)
    v = torch.as_tensor(v_np.reshape(ny, nx), device="cuda")
    if op == "lap5":
        y = nkhip.lap5_apply(v, 1 / h ** 2).cpu().numpy().reshape(-1)
        ref = sh_oracle.lap5(v_np, ny, nx, 1 / h ** 2)
    else:
        y = nkhip.sh13_apply(v, h, r).cpu().numpy().reshape(-1)
        ref = sh_oracle.sh13(v_np, ny, nx, h, r)
    assert np.abs(y - ref).max() <= 1e-13 * max(1.0, np.abs(ref).max())
