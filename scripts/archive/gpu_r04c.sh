#!/bin/bash
# Round 4: the whole GPU suite after the peer-communicator changes, then the world-of-one peer
# slab path under rocprofv3 (kernel trace + stats, then the two counter passes) and the
# communicator A/B at world size 1.
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 900 --timeout-method thread \
  > gpurun_out/r04c_gputest.log 2>&1
rc=$?
tail -5 gpurun_out/r04c_gputest.log
[ $rc -eq 0 ] || exit $rc
bash scripts/profile.sh r04slab --peer-self --steps 3 --warmup 1 --cpu-baseline off --extra off --pmc off \
  > gpurun_out/r04c_prof.log 2>&1 || { tail -20 gpurun_out/r04c_prof.log; exit 1; }
tail -4 gpurun_out/r04c_prof.log
VARIANTS="plain peer peerxk" bash scripts/ab_comm.sh 2
