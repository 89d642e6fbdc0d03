"""GPU: the peer-memory slab communicator (csrc/peer.hip) against the single periodic slab.

Two ways to run the same protocol on one MI355X:
  * a world of one (the rank is its own previous and next neighbour, its halo comes back through
    its own buffer);
  * several PROCESSES on one GPU, the buffers mapped through IPC handles exchanged over a gloo
    torch.distributed group -- the multi-process path the 8-GPU bench runs, minus xGMI.
Several ranks as threads of ONE process are not a supported way to run it (only the abort test
does, with one rank idle): HIP maps the process's streams onto GPU_MAX_HW_QUEUES (4) in-order
hardware queues, so a slab's collective kernel, waiting for a peer slab, can sit in the same
queue ahead of the very launch it waits for.  One process per slab has its own queues.
Parity bar as for the other slab tests: the gathered slabs equal the single-slab step to
1e-8 max(1, |U|) at f_tol = 1e-10 (the decomposition only changes summation order).
"""
import os
import socket
import sys
import threading
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


def test_peer_abort_releases_blocked_rank():
    """nk_comm_abort's contract: rank 1 fails before its step; rank 0, already waiting in a
    collective for it, returns NK_ECOMM (an NKError) within seconds instead of hanging."""
    import nkhip
    N = 64
    comms = nkhip.peer_comms(2, N)
    U0 = np.random.default_rng(1).standard_normal((N, N))
    err = [None]
    done = threading.Event()

    def rank0():
        stream = torch.cuda.Stream()
        try:
            with torch.cuda.stream(stream):
                row0, ny = nkhip.slab_rows(N, 0, 2)
                m = nkhip.SwiftHohenberg(N=N, d=0.625 * N, comm=comms[0], ny_local=ny,
                                         stream=stream)
                m.step(torch.as_tensor(U0[row0:row0 + ny].copy(), device="cuda"))
        except Exception as e:  # noqa: BLE001 - the expected failure
            err[0] = e
        finally:
            done.set()

    t = threading.Thread(target=rank0, daemon=True)
    t0 = time.time()
    t.start()
    time.sleep(2.0)  # rank 0 is inside its first collective by now
    comms[1].abort()
    assert done.wait(60), "rank 0 still blocked 60 s after the abort"
    assert isinstance(err[0], nkhip.NKError), err[0]
    assert time.time() - t0 < 60
    for c in comms:
        c.close()


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
m = nkhip.SwiftHohenberg(N=N, d=0.625 * N, f_tol=1e-10, comm=comm, ny_local=ny)
U = torch.as_tensor(U0[row0:row0 + ny].copy(), device="cuda")
steps = int(os.environ.get("GRID_STEPS", "1"))
for _ in range(steps):
    U = m.step(U)
st = m.last_stats
torch.cuda.synchronize()
np.save(os.path.join(os.environ["OUT_DIR"], f"slab{{rank}}.npy"), U.cpu().numpy())
print(f"rank {{rank}} nit {{st['nit']}} narn {{st['n_arnoldi']}} dev {{st['n_device_steps']}}",
      flush=True)
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
@pytest.mark.parametrize("world,N,steps,xk", [(2, 128, 2, "auto"), (2, 61, 1, "auto"),
                                             (3, 96, 1, "auto"), (4, 128, 1, "auto"),
                                             (8, 256, 1, "auto"), (2, 128, 2, "1"),
                                             (3, 96, 1, "1"), (4, 256, 1, "1")])
def test_peer_processes_match_single_slab(world, N, steps, xk, tmp_path):
    """``world`` processes on one GPU, one slab each, the peer buffers mapped through IPC
    (dmabuf) handles: the gathered slabs equal the single-slab steps.  World 2 has prev == next
    (both halo directions go to one peer); N = 61 takes the point kernel (odd nx); 8 x 256 runs
    the fused Arnoldi step on 32-row slabs with the device-side control.  xk = "1": the fused
    kernel's edge bands run the slab exchange themselves (NKHIP_SLAB_XK=1 forces it although the
    ranks share this GPU: the ranks' grids then wait on each other's edge bands, which always
    progresses -- publishing never waits -- but slowly; "auto" takes the edge + halo kernel)."""
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
    for p, o in zip(procs, outs):
        assert p.returncode == 0, o[-3000:]
    got = np.concatenate([np.load(tmp_path / f"slab{r}.npy") for r in range(world)], axis=0)
    assert np.abs(got - ref).max() <= 1e-8 * max(1.0, np.abs(ref).max()), outs
