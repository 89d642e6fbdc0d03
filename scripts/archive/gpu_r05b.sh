#!/bin/bash
# Round 5: streaming ceilings of this box -- copy variants (scripts/micro/copy_bench.hip) at one
# and four 4096^2 vectors per copy, and the fused kernel's bare march pattern (march_bench.hip).
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 120 scripts/micro/copy_bench 16777216 > gpurun_out/r05b_copy.log 2>&1 || exit 1
timeout -k 10 120 scripts/micro/copy_bench 67108864 >> gpurun_out/r05b_copy.log 2>&1 || exit 1
timeout -k 10 120 scripts/micro/march_bench 16384 > gpurun_out/r05b_march.log 2>&1 || exit 1
timeout -k 10 120 scripts/micro/march_bench 0 >> gpurun_out/r05b_march.log 2>&1 || exit 1
cat gpurun_out/r05b_copy.log gpurun_out/r05b_march.log
