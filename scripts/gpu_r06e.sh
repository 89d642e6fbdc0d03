#!/bin/bash
# Round 6: the alternating march with temporal loads for the band-boundary rows -- correctness
# (march-direction tests), the A/B against the all-down march on 512 .. 4096-row grids (one call),
# the 512-row per-instantiation traffic with it on, and the ARN_OPQ=2 error pattern of the round-5 kernel under the
# bounds-checked ARN_OPQ=2 build (scripts/dbg/opq2_probe.py).
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
O=$PWD/gpurun_out/r06e
mkdir -p "$O"
L=$PWD/iterative-solvers-summer-2020_amd/nkhip
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread \
    tests/test_gpu_fused.py -k "march_direction" > "$O/tests.log" 2>&1 || { tail -30 "$O/tests.log"; exit 1; }
tail -1 "$O/tests.log"
for rep in 1 2; do
  for alt in 0 1; do
    echo "alt=$alt $(NKHIP_ARN_ALT=$alt timeout -k 10 200 python3 scripts/slab_size_probe.py 512 1024 2048 4096 2>/dev/null | tr '\n' ' ')" | tee -a "$O/ab.log"
  done
done
ny=512
export NKHIP_ARN_ALT=1
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d "$O/t$ny" -o t --output-format csv \
    -- python3 scripts/slab_size_probe.py $ny > "$O/t$ny.log" 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d "$O/f$ny" -o f --output-format csv \
    -- python3 scripts/slab_size_probe.py $ny > "$O/f$ny.log" 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d "$O/w$ny" -o w --output-format csv \
    -- python3 scripts/slab_size_probe.py $ny > "$O/w$ny.log" 2>&1 || exit 1
python3 scripts/slab_kernels.py "$O/t$ny/t_kernel_stats.csv" "$O/f$ny/f_counter_collection.csv" \
    "$O/w$ny/w_counter_collection.csv" $ny | tee "$O/kernels_$ny.txt"
unset NKHIP_ARN_ALT
if [ -f "$L/libnkhip_r05_check_opq2.so" ]; then
  for nv in 25 19 30; do
    NV=$nv NKHIP_LIB=$L/libnkhip_r05_check_opq2.so timeout -k 10 120 python3 scripts/dbg/opq2_pattern.py \
        2>/dev/null | grep PATTERN | tee -a "$O/opq2_pattern.log"
  done
fi
