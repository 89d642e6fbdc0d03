"""The N = 8 rank's work with its slab machinery, measured on one GPU: a world-of-one peer-memory
group (the communicator the N > 1 bench uses, its pushed-halo-rows path: the slab's halo rows come
from its own slots, the reduction + all-reduce + control is one launch per Arnoldi step) over an
ny x 4096 slab stepped from default_rng(2020); ms per Arnoldi step and the per-class kernel time
(HIP events on every 8th launch).  Beside scripts/slab_size_probe.py (the plain periodic slab, no
communicator), the difference is the slab path's own cost per Arnoldi step; what it cannot show
is xGMI latency (the peers are this process).
    python3 scripts/slab_peer_probe.py [ny ...]"""
import json
import os
import socket
import sys
import time

import numpy as np
import torch
import torch.distributed as dist

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "iterative-solvers-summer-2020_amd"))
import nkhip  # noqa: E402


def run(comm, ny, nx=4096, warmup=2, steps=4):
    U0 = np.random.default_rng(2020).standard_normal((ny, nx))
    m = nkhip.SwiftHohenberg(N=nx, ny=ny, d=0.625 * nx, comm=comm, ny_local=ny, profile=8)
    a = torch.as_tensor(U0, device="cuda")
    b = torch.empty_like(a)
    for _ in range(warmup):
        m.step(a, out=b)
        a, b = b, a
    m.reset_profile()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    narn = 0
    for _ in range(steps):
        m.step(a, out=b)
        narn += m.last_stats["njvp"]
        a, b = b, a
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    prof = m.kernel_profile()
    m.close()
    per = {k: round(1e3 * v["ms"] / v["timed"], 1) for k, v in prof.items() if v.get("timed")}
    f = prof.get("arnoldi_fused", {})
    gbs = f["timed_bytes"] / (f["ms"] * 1e-3) / 1e9 if f.get("timed") else None
    return {"ny": ny, "ms_per_arnoldi": round(1e3 * dt / max(narn, 1), 4),
            "fused_frac": round(gbs / 8000, 4) if gbs else None, "avg_us": per,
            "launches_per_arnoldi": {k: round(v["launches"] / max(narn, 1), 2)
                                     for k, v in prof.items() if v.get("launches")}}


if __name__ == "__main__":
    with socket.socket() as s_:
        s_.bind(("127.0.0.1", 0))
        port = s_.getsockname()[1]
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1)
    comm = nkhip.PeerComm.from_torch_distributed(max_nx=4096)
    assert comm.selftest(4096) and comm.selftest_push(4096) is not False
    for ny in [int(x) for x in sys.argv[1:]] or [512, 4096]:
        print(json.dumps(run(comm, ny)), flush=True)
    comm.close()
    dist.destroy_process_group()
