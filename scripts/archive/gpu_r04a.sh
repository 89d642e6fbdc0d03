#!/bin/bash
# Round 4, first GPU call: the peer-communicator changes (bounded halo grids, wall-clock wait
# bound, one process per rank), bench.py's self-launch at --gpus 4 on one GPU, and where the
# slab path's runtime blits come from.
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest -x -v --timeout 600 --timeout-method thread \
  tests/test_gpu_peer.py tests/test_gpu_bench.py > gpurun_out/r04a_tests.log 2>&1
rc=$?
tail -25 gpurun_out/r04a_tests.log
[ $rc -eq 0 ] || exit $rc
bash scripts/diag_blits.sh
