#!/bin/bash
# Round 6: why the alternating march barely moved the 512-row traffic.  In one call: the round-5
# library (libnkhip_r05.so, the fused kernel before the logical-row refactor) against this one
# with NKHIP_ARN_ALT 0 / 1, and the streamed loads non-temporal (default) or not (NKHIP_ARN_NT=0:
# whether the halo rows' second read can hit L2 when the first one was a temporal load);
# per-instantiation HBM traffic at 512 rows for ALT=1 NT=0.
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
O=$PWD/gpurun_out/r06c
mkdir -p "$O"
L=$PWD/iterative-solvers-summer-2020_amd/nkhip
for rep in 1 2; do
  for v in r05 a0 a1 a0n a1n; do
    case $v in
      r05) env="NKHIP_LIB=$L/libnkhip_r05.so" ;;
      a0) env="NKHIP_ARN_ALT=0" ;;
      a1) env="NKHIP_ARN_ALT=1" ;;
      a0n) env="NKHIP_ARN_ALT=0 NKHIP_ARN_NT=0" ;;
      a1n) env="NKHIP_ARN_ALT=1 NKHIP_ARN_NT=0" ;;
    esac
    echo "$v $(env $env timeout -k 10 200 python3 scripts/slab_size_probe.py 512 4096 2>/dev/null | tr '\n' ' ')" | tee -a "$O/ab.log"
  done
done
ny=512
export NKHIP_ARN_ALT=1 NKHIP_ARN_NT=0
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d "$O/t$ny" -o t --output-format csv \
    -- python3 scripts/slab_size_probe.py $ny > "$O/t$ny.log" 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d "$O/f$ny" -o f --output-format csv \
    -- python3 scripts/slab_size_probe.py $ny > "$O/f$ny.log" 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d "$O/w$ny" -o w --output-format csv \
    -- python3 scripts/slab_size_probe.py $ny > "$O/w$ny.log" 2>&1 || exit 1
python3 scripts/slab_kernels.py "$O/t$ny/t_kernel_stats.csv" "$O/f$ny/f_counter_collection.csv" \
    "$O/w$ny/w_counter_collection.csv" $ny | tee "$O/kernels_$ny.txt"
# the ARN_OPQ=2 question (scripts/dbg/opq2_probe.py): check + pinned, product + pinned, check
unset NKHIP_ARN_ALT NKHIP_ARN_NT
for lib in check_opq2 opq2 check; do
  for mbox in 1 2; do
    NKHIP_LIB=$L/libnkhip_$lib.so NKHIP_ARN_MBOX=$mbox timeout -k 10 120 python3 scripts/dbg/opq2_probe.py \
        2>/dev/null | tee -a "$O/opq2.log" || echo "{\"lib\": \"$lib\", \"mbox\": $mbox, \"rc\": $?}" | tee -a "$O/opq2.log"
  done
done
