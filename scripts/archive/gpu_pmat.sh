#!/bin/bash
# PMA loop stage timing (NKHIP_PMA_TIMING: per-stage wall clock of the persistent kernel).
set -o pipefail
mkdir -p gpurun_out
NKHIP_PMA_TIMING=1 timeout -k 10 120 python3 scripts/droplet_run.py 2 > gpurun_out/pma_timing.log 2>&1 || exit $?
grep "pma us" gpurun_out/pma_timing.log | tail -n 2
timeout -k 10 600 python -u -m pytest tests/test_gpu_droplet.py tests/test_gpu_mems.py -q -x --timeout 120 \
  --timeout-method thread > gpurun_out/drop_tests.log 2>&1
rc=$?; tail -2 gpurun_out/drop_tests.log; exit $rc
