#!/bin/bash
# Round-4 end state: the whole GPU suite, smoke(), rocprofv3 passes over the default one-GPU
# bench (kernel trace + stats, FETCH_SIZE, WRITE_SIZE), and the default bench line.
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 1000 python3 -u -m pytest tests -m gpu -x -q --timeout 900 --timeout-method thread \
  > gpurun_out/r04q_gputest.log 2>&1
rc=$?
tail -5 gpurun_out/r04q_gputest.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r04q_smoke.log 2>&1 || { tail -5 gpurun_out/r04q_smoke.log; exit 1; }
tail -1 gpurun_out/r04q_smoke.log
bash scripts/profile.sh r04q > gpurun_out/r04q_prof.log 2>&1 || { tail -20 gpurun_out/r04q_prof.log; exit 1; }
tail -3 gpurun_out/r04q_prof.log
timeout -k 10 900 python3 bench.py > gpurun_out/r04q_bench.log 2>&1
rc=$?
tail -c 800 gpurun_out/r04q_bench.log
exit $rc
