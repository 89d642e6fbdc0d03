#!/bin/bash
# Round 4: the whole GPU suite with the stencil passes writing their outputs' edge arrays, then
# the default bench (with the live traffic passes).
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 900 --timeout-method thread \
  > gpurun_out/r04d_gputest.log 2>&1
rc=$?
tail -5 gpurun_out/r04d_gputest.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python3 bench.py --extra off --cpu-baseline off > gpurun_out/r04d_bench.log 2>&1
rc=$?
tail -c 3000 gpurun_out/r04d_bench.log
exit $rc
