#!/bin/bash
# Round 4: pushed halo rows and the FD-JVP's side columns from edge arrays -- the whole GPU
# suite, then the world-of-one slab A/B and the default bench.
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 1000 python3 -u -m pytest tests -m gpu -x -q --timeout 900 --timeout-method thread \
  > gpurun_out/r04e_tests.log 2>&1
rc=$?
tail -15 gpurun_out/r04e_tests.log
[ $rc -eq 0 ] || exit $rc
VARIANTS="plain peer peerex" bash scripts/ab_comm.sh 2 || exit 1
timeout -k 10 600 python3 bench.py --extra off --cpu-baseline off > gpurun_out/r04e_bench.log 2>&1
rc=$?
tail -c 1500 gpurun_out/r04e_bench.log
exit $rc
