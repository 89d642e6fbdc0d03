#!/bin/bash
# Round 4: stencil halos from the pushed slots (epoch-ordered) -- the whole GPU suite, then the
# world-of-one slab A/B.
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 1000 python3 -u -m pytest tests -m gpu -x -q --timeout 900 --timeout-method thread \
  > gpurun_out/r04k_tests.log 2>&1
rc=$?
tail -8 gpurun_out/r04k_tests.log
[ $rc -eq 0 ] || exit $rc
VARIANTS="plain peer peerex" bash scripts/ab_comm.sh 2
