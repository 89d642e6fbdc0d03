#!/bin/bash
# Round 4: shorter edge bands for the pushed-halo prologue -- slab tests, then the A/B.
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 1000 python3 -u -m pytest tests/test_gpu_peer.py tests/test_gpu_bounds.py \
  tests/test_gpu_bench.py tests/test_gpu_fused.py tests/test_gpu_nk.py -x -q --timeout 900 \
  --timeout-method thread > gpurun_out/r04h_tests.log 2>&1
rc=$?
tail -8 gpurun_out/r04h_tests.log
[ $rc -eq 0 ] || exit $rc
VARIANTS="plain peer peerd0 peerd4 peerex" bash scripts/ab_comm.sh 2
