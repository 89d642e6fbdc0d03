#!/bin/bash
# Which multi-process slab cases fail with the fused launch's tail, and after how long.
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
cat > /tmp/w.py <<'PY'
import os, sys, time
import numpy as np
import torch
import torch.distributed as dist
sys.path[:0] = [os.environ["GRAFT_REPO_ROOT"], os.path.join(os.environ["GRAFT_REPO_ROOT"], "iterative-solvers-summer-2020_amd")]
import nkhip
rank, world, N = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"]), int(os.environ["GRID_N"])
torch.cuda.set_device(0)
dist.init_process_group("gloo")
comm = nkhip.PeerComm.from_torch_distributed(max_nx=N)
assert comm.selftest(N)
U0 = np.random.default_rng(2020).standard_normal((N, N))
row0, ny = nkhip.slab_rows(N, rank, world)
m = nkhip.SwiftHohenberg(N=N, d=0.625 * N, comm=comm, ny_local=ny, f_tol=1e-10)
U = torch.as_tensor(U0[row0:row0 + ny].copy(), device="cuda")
t0 = time.time()
try:
    U = m.step(U)
    st = m.last_stats
    print(f"rank {rank} ok {time.time()-t0:.2f}s nit {st['nit']} narn {st['n_arnoldi']} dev {st['n_device_steps']}", flush=True)
except Exception as e:
    print(f"rank {rank} FAIL {time.time()-t0:.2f}s {e}", flush=True)
dist.barrier()
m.close(); comm.close(); dist.destroy_process_group()
PY
run() {  # world N env...
  local W=$1 N=$2; shift 2
  local port=$((29500 + RANDOM % 1000))
  local pids=()
  for r in $(seq 0 $((W - 1))); do
    env "$@" RANK=$r WORLD_SIZE=$W MASTER_ADDR=127.0.0.1 MASTER_PORT=$port GRID_N=$N LOCAL_RANK=0 \
      timeout -k 5 90 python3 /tmp/w.py > gpurun_out/w_$r.log 2>&1 &
    pids+=($!)
  done
  for p in "${pids[@]}"; do wait $p; done
  echo "== W=$W N=$N $*"
  cat gpurun_out/w_*.log | grep -E "^rank" | sort | head -8
  rm -f gpurun_out/w_*.log
}
run 8 256 NKHIP_PEER_TIMEOUT_S=30
run 4 256 NKHIP_PEER_TIMEOUT_S=8
run 8 128 NKHIP_PEER_TIMEOUT_S=8
run 2 256 NKHIP_PEER_TIMEOUT_S=8
run 8 256 NKHIP_PEER_TIMEOUT_S=8 NKHIP_ARN_TAIL=0
exit 0
