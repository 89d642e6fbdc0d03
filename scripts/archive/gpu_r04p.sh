#!/bin/bash
# The fused launch's tail with write-through hand-offs: stage times (probe build), the
# device-control and slab tests (tail forced where the tests force it), one-GPU host loop /
# device control with and without the tail, and the world-of-one peer slab with and without it.
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
NKHIP_ARN_TAIL=1 NKHIP_LIB=$PWD/iterative-solvers-summer-2020_amd/nkhip/libnkhip_tprobe.so timeout -k 10 300 python3 scripts/dbg/tail_probe.py 2>&1 | grep -v amdgpu.ids || exit 1
NKHIP_ARN_TAIL=1 timeout -k 10 900 python3 -u -m pytest tests/test_gpu_fused.py tests/test_gpu_peer.py tests/test_gpu_bounds.py \
  -x -q --timeout 300 --timeout-method thread > gpurun_out/r04p_tests.log 2>&1 || { tail -40 gpurun_out/r04p_tests.log; exit 1; }
tail -2 gpurun_out/r04p_tests.log
bash scripts/ab_env.sh 2 "NKHIP_DEVCTL=0" "NKHIP_DEVCTL=1 NKHIP_ARN_TAIL=1" "NKHIP_DEVCTL=1" || exit 1
VARIANTS="plain peer peert" bash scripts/ab_comm.sh 2
