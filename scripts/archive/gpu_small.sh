#!/bin/bash
# Small-vector Krylov kernels: full -m gpu suite, droplet step timing, bench with the other configs.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread \
  > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python3 scripts/droplet_run.py 5 > gpurun_out/drop_run.log 2>&1 || exit $?
tail -n 2 gpurun_out/drop_run.log
timeout -k 10 600 python bench.py --steps 5 --warmup 1 --cpu-baseline off > gpurun_out/bench_extra.log 2>&1 || exit $?
grep '^{' gpurun_out/bench_extra.log | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); print(d['value'], d['roofline']['frac']); print(json.dumps(d['other_configs']))"
