"""Round 5: why the fused launch's tail stalled with 8 processes on ONE GPU (profiles/r04_tail.md).
Starts P rank processes on device 0 (peer communicator over IPC, one slab each, N x N grid), each
running one device-controlled step with the tail forced (NKHIP_ARN_TAIL=2) on the tail-probe
library (libnkhip_tprobe.so: ARN_TAIL_PROBE, nk_debug_tail_diag) with short peer waits; a rank
whose tail gives up prints what it was waiting for: its own launch's blocks (arrived / total) or
other ranks' all-reduce contributions (the missing ones).
    python3 scripts/dbg/tail8_probe.py <P> [N]"""
import os
import socket
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
PKG = os.path.join(ROOT, "iterative-solvers-summer-2020_amd")

WORKER = r'''
import ctypes as C, os, sys, time
import numpy as np, torch, torch.distributed as dist
sys.path[:0] = [{pkg!r}]
import nkhip
from nkhip import _lib
rank, world, N = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"]), int(os.environ["GRID_N"])
torch.cuda.set_device(0)
dist.init_process_group("gloo")
comm = nkhip.PeerComm.from_torch_distributed(max_nx=N)
row0, ny = nkhip.slab_rows(N, rank, world)
U0 = np.random.default_rng(2020).standard_normal((N, N))
m = nkhip.SwiftHohenberg(N=N, d=0.625 * N, comm=comm, ny_local=ny, f_tol=1e-10)
U = torch.as_tensor(U0[row0:row0 + ny].copy(), device="cuda")
dist.barrier()
t0 = time.time()
msg = "ok"
try:
    for _ in range(int(os.environ.get("STEPS", "1"))):
        U = m.step(U)
    torch.cuda.synchronize()
except Exception as e:
    msg = f"failed: {{e}}"
dt = time.time() - t0
d = (C.c_ulonglong * 8)()
rc = _lib.lib.nk_debug_tail_diag(d)
kind = {{0: "none", 1: "own blocks' arrival", 2: "peer all-reduce"}}.get(int(d[0]), str(d[0]))
miss = [q for q in range(world) if (int(d[3]) >> q) & 1]
print(f"rank {{rank}} {{msg[:90]}} after {{dt:.2f}} s; tail gave up: {{kind}}, arrived {{d[1]}}/{{d[2]}}, "
      f"missing peers {{miss}}, {{d[4] / 100:.0f}} us after the launch's first arrival, "
      f"gave-ups {{d[5]}}; stats {{dict(m.last_stats) if msg == 'ok' else ''}}", flush=True)
os._exit(0)
'''


def main():
    P = int(sys.argv[1])
    N = int(sys.argv[2]) if len(sys.argv) > 2 else 256
    tmp = os.path.join(os.environ.get("TMPDIR", "/tmp"), f"tail8_{os.getpid()}.py")
    with open(tmp, "w") as f:
        f.write(WORKER.format(pkg=PKG))
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    procs = []
    for r in range(P):
        env = dict(os.environ, RANK=str(r), WORLD_SIZE=str(P), MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=str(port), LOCAL_RANK="0", GRID_N=str(N),
                   NKHIP_ARN_TAIL=os.environ.get("NKHIP_ARN_TAIL", "2"),
                   NKHIP_PEER_TIMEOUT_S=os.environ.get("NKHIP_PEER_TIMEOUT_S", "5"),
                   NKHIP_LIB=os.path.join(PKG, "nkhip", "libnkhip_tprobe.so"))
        procs.append(subprocess.Popen([sys.executable, tmp], env=env, stdout=subprocess.PIPE,
                                      stderr=subprocess.STDOUT, text=True))
    for p in procs:
        try:
            out = p.communicate(timeout=120)[0]
        except subprocess.TimeoutExpired:
            p.kill()
            out = p.communicate()[0]
        print(out.strip()[-600:], flush=True)
    os.unlink(tmp)


if __name__ == "__main__":
    main()
