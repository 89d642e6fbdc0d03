#!/bin/bash
# Moving-mesh checks: droplet / PMA2 GPU tests, droplet step timing, the bench's other configs.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_droplet.py tests/test_gpu_mems.py -q -x --timeout 120 \
  --timeout-method thread > gpurun_out/drop_tests.log 2>&1
rc=$?; tail -3 gpurun_out/drop_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python3 scripts/droplet_run.py 6 > gpurun_out/drop_run.log 2>&1 || exit $?
tail -n 3 gpurun_out/drop_run.log | cut -c1-200
if [ "${WITH_BENCH:-0}" = 1 ]; then
  timeout -k 10 600 python bench.py --steps 3 --warmup 1 --cpu-baseline off > gpurun_out/bench_extra.log 2>&1 || exit $?
  grep '^{' gpurun_out/bench_extra.log | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); o=d['other_configs']; print(d['value'], o['config3']['gpu_steps_per_s'], o['pma2']['gpu_steps_per_s'], o['sh_linearised'])"
fi
