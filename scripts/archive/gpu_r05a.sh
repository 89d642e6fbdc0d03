#!/bin/bash
# Round 5, first GPU call: the slab-path correctness work (one-row last bands, pushed-halo-rows
# self-test + fallback, config-5 leg of the N > 1 line) and the fused kernels it touches.
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest tests/test_gpu_peer.py tests/test_gpu_bench.py \
  tests/test_gpu_fused.py tests/test_gpu_bounds.py -m gpu -x -v -k "not config5_16384" \
  --timeout 600 --timeout-method thread > gpurun_out/r05a_tests.log 2>&1
rc=$?
tail -15 gpurun_out/r05a_tests.log
exit $rc
