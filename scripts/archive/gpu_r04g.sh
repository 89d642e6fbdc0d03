#!/bin/bash
# Round 4: single-latency pushed-halo prologue, control state uploaded in-kernel, one-load Gram
# fill -- the whole GPU suite, the world-of-one slab A/B, and device control on / off on one GPU.
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 1000 python3 -u -m pytest tests -m gpu -x -q --timeout 900 --timeout-method thread \
  > gpurun_out/r04g_tests.log 2>&1
rc=$?
tail -15 gpurun_out/r04g_tests.log
[ $rc -eq 0 ] || exit $rc
VARIANTS="plain peer peerex" bash scripts/ab_comm.sh 2 || exit 1
bash scripts/ab_env.sh 1 "NKHIP_DEVCTL=0" "NKHIP_DEVCTL=1" "NKHIP_DEVCTL=0" "NKHIP_DEVCTL=1"
