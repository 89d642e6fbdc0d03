#!/bin/bash
# Round 6: alternating march direction (arnoldi.hip "March direction") -- correctness against the
# all-down march, then the A/B on short slabs and the full grid (slab_size_probe, alternating
# NKHIP_ARN_ALT 0 / 1 in one call), then the per-instantiation traffic at 512 rows with it on.
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
O=$PWD/gpurun_out/r06b
mkdir -p "$O"
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread \
    tests/test_gpu_fused.py -k "march_direction" > "$O/tests.log" 2>&1 || { tail -30 "$O/tests.log"; exit 1; }
tail -2 "$O/tests.log"
for rep in 1 2; do
  for alt in 0 1; do
    echo "alt=$alt $(NKHIP_ARN_ALT=$alt timeout -k 10 200 python3 scripts/slab_size_probe.py 512 1024 4096 2>/dev/null | tr '\n' ' ')" | tee -a "$O/ab.log"
  done
done
ny=512
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d "$O/t$ny" -o t --output-format csv \
    -- python3 scripts/slab_size_probe.py $ny > "$O/t$ny.log" 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d "$O/f$ny" -o f --output-format csv \
    -- python3 scripts/slab_size_probe.py $ny > "$O/f$ny.log" 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d "$O/w$ny" -o w --output-format csv \
    -- python3 scripts/slab_size_probe.py $ny > "$O/w$ny.log" 2>&1 || exit 1
python3 scripts/slab_kernels.py "$O/t$ny/t_kernel_stats.csv" "$O/f$ny/f_counter_collection.csv" \
    "$O/w$ny/w_counter_collection.csv" $ny | tee "$O/kernels_$ny.txt"
