"""Stage times of the control launch of the pushed slab path (arn_reduce_allreduce_ctl_kernel,
ARN_CTL_PROBE build: NKHIP_LIB=.../libnkhip_cprobe.so): a world-of-one peer-memory group over an
ny x 4096 slab (scripts/slab_peer_probe.py's setup), a few steps, then the summed wall-clock ticks
(100 MHz) of each stage per launch.
    NKHIP_LIB=... python3 scripts/dbg/ctl_probe.py [ny]"""
import ctypes as C
import os
import socket
import sys

import numpy as np
import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "iterative-solvers-summer-2020_amd"))
import nkhip  # noqa: E402
from nkhip import _lib  # noqa: E402

ny = int(sys.argv[1]) if len(sys.argv) > 1 else 512
nx = 4096
with socket.socket() as s_:
    s_.bind(("127.0.0.1", 0))
    port = s_.getsockname()[1]
dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1)
comm = nkhip.PeerComm.from_torch_distributed(max_nx=nx)
m = nkhip.SwiftHohenberg(N=nx, ny=ny, d=0.625 * nx, comm=comm, ny_local=ny, profile=0)
a = torch.as_tensor(np.random.default_rng(2020).standard_normal((ny, nx)), device="cuda")
b = torch.empty_like(a)
out = (C.c_ulonglong * 8)()
m.step(a, out=b)
a, b = b, a
assert _lib.lib.nk_debug_ctl_probe(out) == 0
for _ in range(3):
    m.step(a, out=b)
    a, b = b, a
assert _lib.lib.nk_debug_ctl_probe(out) == 0
cnt = max(out[0], 1)
names = ["first entry -> last block counted in", "-> values collected (LDS)", "-> all-reduced",
         "-> control done", "(first entry -> last block's entry)"]
print(f"ny {ny} launches {out[0]}")
for i, nm in enumerate(names):
    print(f"{nm:40s} {out[i + 1] / cnt / 100:.2f} us", flush=True)
m.close()
comm.close()
dist.destroy_process_group()
