#!/bin/bash
# A/B of the slab edge kernel (arnoldi_edge: u on a slab's 4 edge rows) through the RCCL self-halo
# bench, alternating two library builds inside one call (box noise):
#   bash scripts/edge_ab.sh <variant>     (variant: nkhip/libnkhip_<variant>.so against libnkhip.so)
set -o pipefail
mkdir -p gpurun_out
L=$PWD/iterative-solvers-summer-2020_amd/nkhip
for rep in 1 2; do
  for v in "$1" A; do
    lib=$L/libnkhip_$v.so; [ "$v" = A ] && lib=$L/libnkhip.so
    NKHIP_LIB=$lib timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 \
      --master-addr 127.0.0.1 --master-port 29517 bench.py --rccl-self --steps 4 --warmup 1 \
      --cpu-baseline off --extra off > gpurun_out/edge_ab_$v.log 2>&1 || exit $?
    grep '^{' gpurun_out/edge_ab_$v.log | python3 -c "
import sys, json
r = json.loads(sys.stdin.readline()); k = r['kernels']
print('$rep $v', r['value'], 'edge', k['arnoldi_edge']['avg_us'], 'halo', k['halo']['avg_us'],
      'fused', k['arnoldi_fused']['avg_us'])" || exit $?
  done
done
