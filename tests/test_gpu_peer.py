"""GPU: the peer-memory slab communicator (csrc/peer.hip) against the single periodic slab.

Two ways to run the same protocol on one MI355X:
  * a world of one (the rank is its own previous and next neighbour, its halo comes back through
    its own buffer);
  * several PROCESSES on one GPU, the buffers mapped through IPC handles exchanged over a gloo
    torch.distributed group -- the multi-process path the 8-GPU bench runs, minus xGMI.
Several ranks as threads of ONE process are refused (nk_comm_peer_connect: NK_EINVAL): HIP maps
the process's streams onto GPU_MAX_HW_QUEUES (4) in-order hardware queues, so a slab's
collective kernel, waiting for a peer slab, could sit in the same queue ahead of the very launch
it waits for.  One process per slab has its own queues.
Parity bar as for the other slab tests: the gathered slabs equal the single-slab step to
1e-8 max(1, |U|) at f_tol = 1e-10 (the decomposition only changes summation order).
"""
import os
import socket
import sys
import time

import numpy as np
import pytest
import torch

from conftest import PKG, ROOT

pytestmark = pytest.mark.gpu


def _single(N, U0, **kw):
    import nkhip
    m = nkhip.SwiftHohenberg(N=N, d=0.625 * N, f_tol=1e-10, **kw)
    ref = m.step(torch.as_tensor(U0, device="cuda")).cpu().numpy()
    m.close()
    return ref


@pytest.mark.parametrize("xk", ["0", "2"])
def test_peer_world1_matches_single_slab(xk, monkeypatch):
    """A world of one through the peer communicator: the edge + halo kernel (xk 0) and the fused
    kernel's in-kernel slab exchange (NKHIP_SLAB_XK=2; the rank is its own neighbour)."""
    monkeypatch.setenv("NKHIP_SLAB_XK", xk)
    import nkhip
    N = 96
    U0 = np.random.default_rng(2020).standard_normal((N, N))
    ref = _single(N, U0)
    (comm,) = nkhip.peer_comms(1, N)
    try:
        assert comm.selftest(N)
        m = nkhip.SwiftHohenberg(N=N, d=0.625 * N, f_tol=1e-10, comm=comm, ny_local=N)
        got = m.step(torch.as_tensor(U0, device="cuda")).cpu().numpy()
        m.close()
    finally:
        comm.close()
    assert np.abs(got - ref).max() <= 1e-8 * max(1.0, np.abs(ref).max())


# ---------------------------------------------------------------------------------------------
# several processes on one GPU
# ---------------------------------------------------------------------------------------------
_WORKER = r'''
import os, sys
import numpy as np
import torch
import torch.distributed as dist
sys.path[:0] = [{root!r}, {pkg!r}]
import nkhip
rank, world, N = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"]), int(os.environ["GRID_N"])
torch.cuda.set_device(0)
dist.init_process_group("gloo")
comm = nkhip.PeerComm.from_torch_distributed(max_nx=N)
assert comm.selftest(N), "nk_comm_selftest failed"  # the bench's check before it trusts the group
U0 = np.random.default_rng(2020).standard_normal((N, N))
row0, ny = nkhip.slab_rows(N, rank, world)
ftol = os.environ.get("GRID_FTOL", "1e-10")
kw = {{}} if ftol == "default" else {{"f_tol": float(ftol)}}
m = nkhip.SwiftHohenberg(N=N, d=0.625 * N, comm=comm, ny_local=ny, **kw)
U = torch.as_tensor(U0[row0:row0 + ny].copy(), device="cuda")
del U0
steps = int(os.environ.get("GRID_STEPS", "1"))
for _ in range(steps):
    U = m.step(U)
st = m.last_stats
torch.cuda.synchronize()
np.save(os.path.join(os.environ["OUT_DIR"], f"slab{{rank}}.npy"), U.cpu().numpy())
print(f"rank {{rank}} nit {{st['nit']}} narn {{st['n_arnoldi']}} dev {{st['n_device_steps']}} "
      f"status {{st['status']}}", flush=True)
dist.barrier()
m.close()
comm.close()
dist.destroy_process_group()
'''


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.timeout(300)
@pytest.mark.parametrize("world,N,steps,xk,tail", [
    (2, 128, 2, "auto", None), (2, 61, 1, "auto", None), (3, 96, 1, "auto", None),
    (4, 128, 1, "auto", None), (8, 256, 1, "auto", None), (2, 200, 1, "auto", None),
    (2, 200, 1, "1", None), (2, 128, 2, "1", None),
    (3, 96, 1, "1", None), (4, 256, 1, "1", None), (2, 128, 2, "auto", "2"),
    (4, 256, 1, "auto", "2")])
def test_peer_processes_match_single_slab(world, N, steps, xk, tail, tmp_path):
    """``world`` processes on one GPU, one slab each, the peer buffers mapped through IPC
    (dmabuf) handles: the gathered slabs equal the single-slab steps.  World 2 has prev == next
    (both halo directions go to one peer); N = 61 takes the point kernel (odd nx); 8 x 256 runs
    the fused Arnoldi step on 32-row slabs with the device-side control.  xk = "1": the fused
    kernel's edge bands run the slab exchange themselves (NKHIP_SLAB_XK=1 forces it although the
    ranks share this GPU: the ranks' grids then wait on each other's edge bands, which always
    progresses -- publishing never waits -- but slowly; "auto" takes the edge + halo kernel).
    tail = "2": the fused launches' tails run the reduction, the all-reduce and the control
    although the ranks share this GPU (NKHIP_ARN_TAIL=2; by default they do so only with one
    rank per GPU).  N = 200 on 2 ranks: 100-row slabs whose band plan ends in a one-row band, so
    the band before it also reads the halo rows ny, ny+1 (it computes / waits for them itself)."""
    import subprocess
    U0 = np.random.default_rng(2020).standard_normal((N, N))
    import nkhip
    m = nkhip.SwiftHohenberg(N=N, d=0.625 * N, f_tol=1e-10)
    U = torch.as_tensor(U0, device="cuda")
    for _ in range(steps):
        U = m.step(U)
    ref = U.cpu().numpy()
    m.close()
    script = tmp_path / "worker.py"
    script.write_text(_WORKER.format(root=ROOT, pkg=PKG))
    port = _free_port()
    procs = []
    for r in range(world):
        env = dict(os.environ, RANK=str(r), WORLD_SIZE=str(world), MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=str(port), GRID_N=str(N), GRID_STEPS=str(steps),
                   OUT_DIR=str(tmp_path), LOCAL_RANK="0")
        if xk != "auto":
            env["NKHIP_SLAB_XK"] = xk
        if tail is not None:
            env["NKHIP_ARN_TAIL"] = tail
        procs.append(subprocess.Popen([sys.executable, str(script)], env=env,
                                      stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True))
    outs = []
    for p in procs:
        try:
            outs.append(p.communicate(timeout=240)[0])
        except subprocess.TimeoutExpired:
            for q in procs:
                q.kill()
            raise
    assert all(p.returncode == 0 for p in procs), "\n".join(
        f"--- rank {r} rc {p.returncode}\n{o[-1500:]}" for r, (p, o) in enumerate(zip(procs, outs)))
    got = np.concatenate([np.load(tmp_path / f"slab{r}.npy") for r in range(world)], axis=0)
    assert np.abs(got - ref).max() <= 1e-8 * max(1.0, np.abs(ref).max()), outs


def _run_workers(tmp_path, body, world, extra_env=None, timeout=240):
    """``world`` processes of the worker ``body`` on this GPU (gloo side channel); returns their
    outputs after asserting every exit code is 0."""
    import subprocess
    script = tmp_path / "worker.py"
    script.write_text(body.format(root=ROOT, pkg=PKG))
    port = _free_port()
    procs = []
    for r in range(world):
        env = dict(os.environ, RANK=str(r), WORLD_SIZE=str(world), MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=str(port), OUT_DIR=str(tmp_path), LOCAL_RANK="0",
                   **(extra_env or {}))
        procs.append(subprocess.Popen([sys.executable, str(script)], env=env,
                                      stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True))
    outs = []
    for p in procs:
        try:
            outs.append(p.communicate(timeout=timeout)[0])
        except subprocess.TimeoutExpired:
            for q in procs:
                q.kill()
            raise
    for p, o in zip(procs, outs):
        assert p.returncode == 0, o[-3000:]
    return outs


_ABORT_WORKER = r"""
import os, sys, time
import numpy as np
import torch
import torch.distributed as dist
sys.path[:0] = [{root!r}, {pkg!r}]
import nkhip
rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
torch.cuda.set_device(0)
dist.init_process_group("gloo")
N = 64
comm = nkhip.PeerComm.from_torch_distributed(max_nx=N)
dist.barrier()
if rank == 1:
    time.sleep(2.0)  # rank 0 is inside its first collective by now
    comm.abort()
    print("rank 1 aborted", flush=True)
else:
    U0 = np.random.default_rng(1).standard_normal((N, N))
    row0, ny = nkhip.slab_rows(N, 0, world)
    t0 = time.time()
    try:
        m = nkhip.SwiftHohenberg(N=N, d=0.625 * N, comm=comm, ny_local=ny)
        m.step(torch.as_tensor(U0[row0:row0 + ny].copy(), device="cuda"))
        raise SystemExit("rank 0 stepped although its peer aborted")
    except nkhip.NKError as e:
        dt = time.time() - t0
        assert dt < 60, dt
        print(f"rank 0 released after {{dt:.1f}} s: {{e}}", flush=True)
torch.cuda.synchronize()
comm.close()
"""


@pytest.mark.parametrize("N", [128, 100])
def test_peer_world1_push_matches_exchange_bitwise(N, monkeypatch):
    """The pushed-halo-rows path (default: every producer writes its edge rows into the
    neighbours' halo slots, the fused kernel's edge bands form u on the halo rows from them) and
    the edge + halo exchange kernel (NKHIP_SLAB_PUSH=0) give the same bits: the halo rows are
    the same update sums in the same order.  N = 100: a band plan ending in a one-row band."""
    import nkhip
    U0 = np.random.default_rng(7).standard_normal((N, N))
    out = {}
    for mode in ("1", "0"):
        monkeypatch.setenv("NKHIP_SLAB_PUSH", mode)
        (comm,) = nkhip.peer_comms(1, N)
        try:
            m = nkhip.SwiftHohenberg(N=N, d=0.625 * N, f_tol=1e-10, comm=comm, ny_local=N,
                                     profile=1)
            U = torch.as_tensor(U0, device="cuda")
            for _ in range(2):
                U = m.step(U)
            out[mode] = (U.cpu().numpy(), dict(m.last_stats), m.kernel_profile())
            m.close()
        finally:
            comm.close()
    assert np.array_equal(out["1"][0], out["0"][0])
    assert out["1"][1]["nit"] == out["0"][1]["nit"]
    # push mode: no slab edge kernel, the pushes instead; exchange mode: the edge kernel
    assert out["1"][2].get("arnoldi_edge", {}).get("launches", 0) == 0
    assert out["1"][2]["halo_push"]["launches"] > 0
    assert out["0"][2]["arnoldi_edge"]["launches"] > 0


@pytest.mark.timeout(200)
def test_peer_abort_releases_blocked_rank(tmp_path):
    """nk_comm_abort's contract, across processes: rank 1 fails before its step and aborts;
    rank 0, already waiting in a collective for it, gets NK_ECOMM (an NKError) within seconds
    instead of hanging -- the abort word travels through the IPC-mapped buffer."""
    outs = _run_workers(tmp_path, _ABORT_WORKER, 2, timeout=150)
    assert "released" in outs[0] and "aborted" in outs[1], outs


def test_peer_threads_in_one_process_refused():
    """Two ranks of one group in one process: refused at connect (one process per rank)."""
    import nkhip
    with pytest.raises(ValueError):
        nkhip.peer_comms(2, 64)
    a = nkhip.PeerComm.create(0, 2, 64)
    b = nkhip.PeerComm.create(1, 2, 64)
    try:
        with pytest.raises(nkhip.NKError):
            a.connect([a.blob, b.blob])
    finally:
        a.close()
        b.close()


_WIDE_WORKER = r"""
import os, sys
import torch
import torch.distributed as dist
sys.path[:0] = [{root!r}, {pkg!r}]
import nkhip
torch.cuda.set_device(0)
dist.init_process_group("gloo")
NX = int(os.environ["WIDE_NX"])
comm = nkhip.PeerComm.from_torch_distributed(max_nx=NX)
for _ in range(3):
    assert comm.selftest(NX), "nk_comm_selftest failed"
torch.cuda.synchronize()
dist.barrier()
comm.close()
print("ok", flush=True)
"""


@pytest.mark.timeout(200)
def test_peer_wide_rows_shared_gpu(tmp_path):
    """4 processes on this GPU, 16384-column rows: the halo kernel's grid is capped
    (kHaloMaxBlocks) and strides over the row, so it always fits the GPU as a whole although
    every block waits for flags the last block publishes."""
    outs = _run_workers(tmp_path, _WIDE_WORKER, 4, {"WIDE_NX": "16384"}, timeout=150)
    assert all("ok" in o for o in outs), outs


@pytest.mark.timeout(900)
def test_config5_16384_eight_processes(tmp_path):
    """BASELINE config 5 through the multi-process path the 8-GPU bench runs: a 16384^2 grid as 8
    row slabs in 8 PROCESSES on this GPU (a ~16 GB workspace pool each, ~130 GB together), the
    peer-memory communicator mapped through IPC with its self-test at the full row width, one
    default-f_tol FD step from default_rng(2020) under the device-side control.  Every rank
    reports the same Newton count; the gathered state is a root of the oracle residual over the
    whole grid (sh_scipy_nk.py:47-49) and equals the same step solved as ONE 16384^2 slab to the
    tolerance's scale (as test_gpu_nk.py::test_config5_16384_eight_slabs with loopback slabs)."""
    from test_gpu_nk import _residual_rows
    import nkhip
    N, P = 16384, 8
    outs = _run_workers(tmp_path, _WORKER, P, {"GRID_N": str(N), "GRID_STEPS": "1",
                                               "GRID_FTOL": "default"}, timeout=700)
    nits = {int(o.split(" nit ")[1].split()[0]) for o in outs}
    assert len(nits) == 1 and all(" status 0" in o for o in outs), outs
    U1 = np.concatenate([np.load(tmp_path / f"slab{r}.npy") for r in range(P)], axis=0)
    U0 = np.random.default_rng(2020).standard_normal((N, N))
    assert _residual_rows(U1, U0, 0.625, 0.01, 0.2, 1.0) <= 1.01 * np.finfo(float).eps ** (1 / 3)
    m = nkhip.SwiftHohenberg(N=N, d=0.625 * N)
    Us = m.step(torch.as_tensor(U0, device="cuda")).cpu().numpy()
    nit1 = m.last_stats["nit"]
    m.close()
    torch.cuda.empty_cache()
    assert abs(nit1 - nits.pop()) <= 1
    assert float(np.abs(U1 - Us).max()) <= 1e-5 * max(1.0, float(np.abs(Us).max()))


_PUSH_WORKER = r"""
import os, sys
import torch
import torch.distributed as dist
sys.path[:0] = [{root!r}, {pkg!r}]
import nkhip
torch.cuda.set_device(0)
dist.init_process_group("gloo")
NX = int(os.environ["WIDE_NX"])
comm = nkhip.PeerComm.from_torch_distributed(max_nx=NX)
res = [comm.selftest_push(NX) for _ in range(2)]
_, ny = nkhip.slab_rows(64, int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"]))
m = nkhip.SwiftHohenberg(N=64, d=40.0, comm=comm, ny_local=ny)
held = comm.selftest_push(NX)  # the stepper holds the slots: nothing to check, on every rank
m.close()
after = comm.selftest_push(NX)
torch.cuda.synchronize()
dist.barrier()
comm.close()
print(f"push {{res}} held {{held}} after {{after}}", flush=True)
"""


@pytest.mark.timeout(200)
@pytest.mark.parametrize("world,brk", [(1, None), (3, None), (2, "1")])
def test_peer_push_selftest(world, brk, tmp_path):
    """nk_comm_selftest_push -- the pushed-halo-rows protocol as the solver runs it (push into
    the neighbours' slots, no flag, one all-reduce, read back in a kernel, host check): passes on
    1 and 3 processes; with rank 1 pushing wrong rows (NKHIP_PEER_SELFTEST_BREAK_PUSH=1) its
    neighbour (rank 0) fails it; while a stepper holds the slots it is skipped on every rank."""
    env = {"WIDE_NX": "4096"}
    if brk is not None:
        env["NKHIP_PEER_SELFTEST_BREAK_PUSH"] = brk
    outs = _run_workers(tmp_path, _PUSH_WORKER, world, env, timeout=150)
    for r, o in enumerate(outs):
        want = "[False, False]" if (brk is not None and r == 0) else "[True, True]"
        assert f"push {want} held None after" in o, (r, o)
