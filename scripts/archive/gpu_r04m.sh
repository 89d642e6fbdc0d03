#!/bin/bash
# Vector-pair fused layout: the two lag rows in registers (ARN_RLAG) against LDS, isolated
# fused-kernel microbenchmark at 4096^2 (scripts/arnoldi_bench.py), alternating libraries.
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
NVS=${1:-19,20,21,22,23,24}
shift || true
bash scripts/arn_ab.sh "$NVS" A "$@"
