#!/bin/bash
# The fused launch's tail (reduction + control in its last blocks): the device-control and slab
# tests, then the one-GPU host loop / device control with and without the tail, and the
# world-of-one peer slab with and without it.
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest tests/test_gpu_fused.py tests/test_gpu_peer.py tests/test_gpu_bounds.py \
  -x -v --timeout 300 --timeout-method thread > gpurun_out/r04o_tests.log 2>&1 || { tail -40 gpurun_out/r04o_tests.log; exit 1; }
tail -3 gpurun_out/r04o_tests.log
bash scripts/ab_env.sh 2 "NKHIP_DEVCTL=0" "NKHIP_DEVCTL=1" "NKHIP_DEVCTL=1 NKHIP_ARN_TAIL=0" || exit 1
VARIANTS="plain peer peernt" bash scripts/ab_comm.sh 2
