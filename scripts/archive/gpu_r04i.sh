#!/bin/bash
# Round 4 state: the whole GPU suite, the world-of-one slab path with pushed halo rows under
# rocprofv3 (trace + the two counter passes), and the default bench with its live traffic passes.
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 1000 python3 -u -m pytest tests -m gpu -x -q --timeout 900 --timeout-method thread \
  > gpurun_out/r04i_gputest.log 2>&1
rc=$?
tail -5 gpurun_out/r04i_gputest.log
[ $rc -eq 0 ] || exit $rc
bash scripts/profile.sh r04slabp --peer-self --steps 3 --warmup 1 --cpu-baseline off --extra off --pmc off \
  > gpurun_out/r04i_prof.log 2>&1 || { tail -20 gpurun_out/r04i_prof.log; exit 1; }
tail -3 gpurun_out/r04i_prof.log
timeout -k 10 900 python3 bench.py > gpurun_out/r04i_bench.log 2>&1
rc=$?
tail -c 600 gpurun_out/r04i_bench.log
exit $rc
