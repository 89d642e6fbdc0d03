#!/bin/bash
# Moving-mesh checks: droplet / PMA2 GPU tests, then the droplet step timing.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_droplet.py tests/test_gpu_mems.py -q -x --timeout 120 \
  --timeout-method thread > gpurun_out/drop_tests.log 2>&1
rc=$?; tail -3 gpurun_out/drop_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python3 scripts/droplet_run.py 6 > gpurun_out/drop_run.log 2>&1 || exit $?
tail -n 3 gpurun_out/drop_run.log | cut -c1-60
