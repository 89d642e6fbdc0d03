#!/bin/bash
# Round 5: short slabs -- band height floor (NKHIP_ARN_MIN_RY) at 512 / 1024 rows.
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for rep in 1 2; do
  for ry in 8 64 128; do
    echo "min_ry=$ry $(NKHIP_ARN_MIN_RY=$ry timeout -k 10 200 python3 scripts/slab_size_probe.py 512 1024 2>/dev/null | tr '\n' ' ')"
  done
done
