"""CPU, world_size 2 and 3 over gloo: the row-slab decomposition reproduces the single-slab oracle.

Checks the halo protocol (posting order identical to libnkhip's RCCL halo, csrc/comm.cpp) and the
sum/max all-reduce pattern of the distributed Newton-Krylov loop, on CPU processes.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from conftest import PKG, ROOT, load_golden


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, ny, nx, q):
    import sys
    for p in (ROOT, PKG):
        if p not in sys.path:
            sys.path.insert(0, p)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from nkhip.dist import slab_rows  # noqa: E402 (pure arithmetic, no GPU)
        from oracle import sh_oracle, slab_oracle
        h, r, k, g = 0.625, 0.01, 0.2, 1.0
        rng = np.random.default_rng(11)
        U = rng.standard_normal((ny, nx))
        Uo = rng.standard_normal((ny, nx))
        row0, nloc = slab_rows(ny, rank, world)
        u = torch.from_numpy(U[row0:row0 + nloc].copy())
        uo = torch.from_numpy(Uo[row0:row0 + nloc].copy())
        lo, hi = slab_oracle.halo_exchange(u)
        # the halo rows are the periodic neighbours' rows
        assert np.array_equal(lo.numpy(), U[[(row0 - 2) % ny, (row0 - 1) % ny]])
        assert np.array_equal(hi.numpy(), U[[(row0 + nloc) % ny, (row0 + nloc + 1) % ny]])
        Lu = slab_oracle.sh13_slab(u, lo, hi, h, r)
        ref = sh_oracle.sh13(U.reshape(-1), ny, nx, h, r).reshape(ny, nx)
        err_L = float(np.abs(Lu.numpy() - ref[row0:row0 + nloc]).max())
        F = slab_oracle.residual_slab(u, slab_oracle.halo_exchange(uo), (lo, hi), uo, h, r, k, g)
        Fg = slab_oracle.gather_rows(F, ny).numpy()
        Fref = sh_oracle.residual(U.reshape(-1), Uo.reshape(-1), ny, nx, h, r, k, g).reshape(ny, nx)
        err_F = float(np.abs(Fg - Fref).max() / np.abs(Fref).max())
        sums, maxes = slab_oracle.allreduce_sum_max([float((F * F).sum())],
                                                    [float(F.abs().max())])
        err_n2 = abs(sums[0] - float((Fref * Fref).sum())) / float((Fref * Fref).sum())
        err_mx = abs(maxes[0] - float(np.abs(Fref).max()))
        q.put((rank, err_L, err_F, err_n2, err_mx))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,ny,nx", [(2, 64, 48), (3, 61, 40), (2, 4, 8)])
def test_slab_decomposition_matches_global(world, ny, nx):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, ny, nx, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, err_L, err_F, err_n2, err_mx in res:
        assert err_L < 1e-11, (rank, err_L)
        assert err_F < 1e-13, (rank, err_F)
        assert err_n2 < 1e-13 and err_mx == 0.0


def test_golden_fixture_present_for_gpu_box():
    # /root/reference does not exist on the GPU box: everything the GPU tier checks against is here
    z = load_golden("nk_n64_h0625_tight")
    assert z["traj"].shape == (2, 64 * 64)
