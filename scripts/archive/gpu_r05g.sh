#!/bin/bash
# Round 5 state: the whole GPU suite, smoke(), rocprofv3 passes over the default one-GPU bench
# (kernel trace + stats, FETCH_SIZE, WRITE_SIZE), the default bench line and the driver's window.
set -u
TAG=${1:-r05g}
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 1000 python3 -u -m pytest tests -m gpu -x -q --timeout 900 --timeout-method thread \
  > gpurun_out/${TAG}_gputest.log 2>&1
rc=$?
tail -5 gpurun_out/${TAG}_gputest.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/${TAG}_smoke.log 2>&1 || { tail -5 gpurun_out/${TAG}_smoke.log; exit 1; }
tail -1 gpurun_out/${TAG}_smoke.log
bash scripts/profile.sh $TAG > gpurun_out/${TAG}_prof.log 2>&1 || { tail -20 gpurun_out/${TAG}_prof.log; exit 1; }
tail -3 gpurun_out/${TAG}_prof.log
timeout -k 10 900 python3 bench.py > gpurun_out/${TAG}_bench.log 2>&1 || { tail -c 1500 gpurun_out/${TAG}_bench.log; exit 1; }
tail -c 600 gpurun_out/${TAG}_bench.log
timeout -k 10 600 python3 bench.py --steps 20 --warmup 5 --cpu-baseline off --extra off > gpurun_out/${TAG}_bench_w20.log 2>&1 || { tail -c 1500 gpurun_out/${TAG}_bench_w20.log; exit 1; }
python3 -c "
import json; d=json.loads([l for l in open('gpurun_out/${TAG}_bench_w20.log') if l.startswith('{')][-1])
print('window 6-25:', d['value'], d['ms_per_arnoldi_step'], d['roofline']['frac'], d['jvp_roofline']['frac'])"
timeout -k 10 600 python3 scripts/slab_size_probe.py > gpurun_out/${TAG}_slabsize.log 2>&1 && cat gpurun_out/${TAG}_slabsize.log
timeout -k 10 500 bash scripts/arn_ab.sh 8,16,19,20,22,24,28,35 A base > gpurun_out/${TAG}_ab.log 2>&1 && cat gpurun_out/${TAG}_ab.log
