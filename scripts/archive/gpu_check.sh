#!/bin/bash
# Full -m gpu suite, then the headline bench A/B of the mailbox (alternating runs).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread \
  > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -4 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
BENCH_STEPS=${BENCH_STEPS:-10} bash scripts/bench_ab.sh "off:NKHIP_ARN_MBOX=0" "on:NKHIP_ARN_MBOX=1"
