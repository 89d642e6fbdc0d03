#!/bin/bash
# Rows in flight of the vector-pair layout (tuning builds, NKHIP_ARN_PF), mailbox on; and the
# RCCL-slab mailbox test.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_nk.py -x -q --timeout 120 --timeout-method thread \
  -k "rccl" > gpurun_out/rccl_mb.log 2>&1
rc=$?; tail -3 gpurun_out/rccl_mb.log; [ $rc -eq 0 ] || exit $rc
for nv in 24 32; do
  bash scripts/arn_ab.sh $nv t$nv:NKHIP_ARN_PF=1 t$nv:NKHIP_ARN_PF=2 t$nv:NKHIP_ARN_PF=3 || exit $?
done
