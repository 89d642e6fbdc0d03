#!/bin/bash
# Mailbox bring-up, step by step: the plain-path solver test that faulted, then the mailbox
# kernel tests (every basis length), then the mailbox solver tests.  Stops at the first failure.
set -o pipefail
mkdir -p gpurun_out
run() {  # run <name> <timeout> <pytest -k expr>
  timeout -k 10 $2 python -u -m pytest tests/test_gpu_fused.py -x -q -s --timeout 120 \
    --timeout-method thread -k "$3" > gpurun_out/$1.log 2>&1
  local rc=$?; echo "== $1 rc=$rc"; tail -4 gpurun_out/$1.log; return $rc
}
NKHIP_LAUNCH_LOG=gpurun_out/launch.log run plain 200 "test_edges_identical_solve" || exit $?
run mbk 300 "test_fused_kernel_mailbox" || exit $?
run mbs 300 "test_mailbox_solve" || exit $?
