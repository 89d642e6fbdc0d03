#!/bin/bash
# Round 6: where a short slab's fused pass loses -- per-instantiation durations and HBM traffic of
# the fused Arnoldi kernel on a 512 x 4096 periodic slab (the N = 8 strong-scaling rank) beside
# the full 4096 x 4096 grid, from scripts/slab_size_probe.py under rocprofv3.
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
O=$PWD/gpurun_out/r06a
mkdir -p "$O"
for ny in 512 4096; do
  timeout -k 10 240 rocprofv3 --kernel-trace --stats -d "$O/t$ny" -o t --output-format csv \
      -- python3 scripts/slab_size_probe.py $ny > "$O/t$ny.log" 2>&1 || exit 1
  tail -n 1 "$O/t$ny.log"
  timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d "$O/f$ny" -o f --output-format csv \
      -- python3 scripts/slab_size_probe.py $ny > "$O/f$ny.log" 2>&1 || exit 1
  timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d "$O/w$ny" -o w --output-format csv \
      -- python3 scripts/slab_size_probe.py $ny > "$O/w$ny.log" 2>&1 || exit 1
  python3 scripts/slab_kernels.py "$O/t$ny/t_kernel_stats.csv" "$O/f$ny/f_counter_collection.csv" \
      "$O/w$ny/w_counter_collection.csv" $ny | tee "$O/kernels_$ny.txt"
done
