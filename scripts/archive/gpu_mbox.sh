#!/bin/bash
# Mailbox bring-up: kernel parity tests, kernel-level A/B (packed halo / mailbox / recompute),
# headline-bench A/B.  Stops at the first failing step.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_fused.py -x -q --timeout 120 --timeout-method thread \
  -k "${MBOX_K:-mailbox}" > gpurun_out/mbox_tests.log 2>&1
rc=$?; tail -5 gpurun_out/mbox_tests.log; [ $rc -eq 0 ] || exit $rc
bash scripts/arn_ab.sh ${MBOX_NVS:-4,12,18,19,24,30,35} A:NKHIP_ARN_MBOX=0 A:NKHIP_ARN_MBOX=1 A:NKHIP_ARN_MBOX=2 || exit $?
BENCH_STEPS=${BENCH_STEPS:-5} bash scripts/bench_ab.sh "off:NKHIP_ARN_MBOX=0" "on:NKHIP_ARN_MBOX=1"
