#!/bin/bash
# Round 4: the bench self-launch test, config 5 as 8 processes on one GPU, and where the slab
# path's runtime blits come from.
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 1000 python3 -u -m pytest -x -v --timeout 900 --timeout-method thread \
  tests/test_gpu_bench.py tests/test_gpu_peer.py::test_config5_16384_eight_processes \
  tests/test_gpu_capi.py tests/test_gpu_droplet.py::test_ten_full_steps_every_step \
  > gpurun_out/r04b_tests.log 2>&1
rc=$?
tail -25 gpurun_out/r04b_tests.log
[ $rc -eq 0 ] || exit $rc
bash scripts/diag_blits.sh
