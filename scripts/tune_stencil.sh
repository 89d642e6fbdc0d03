#!/bin/bash
# A/B the stencil launch geometry (env overrides read by stencil.hip) on the kernel microbench.
for cfg in "4 32 2048" "4 64 1024" "8 64 2048" "16 128 1024" "2 8 8192" "1 4 16384"; do
  set -- $cfg
  echo "== RY_MIN=$1 RY_MAX=$2 BLOCKS=$3"
  NKHIP_RY_MIN=$1 NKHIP_RY_MAX=$2 NKHIP_BLOCKS=$3 timeout -k 10 120 python scripts/kernel_bench.py 1024 4096 || exit $?
done
