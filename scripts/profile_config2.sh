#!/bin/bash
# Kernel-only rocprofv3 trace of BASELINE config 2 (1024^2 5-point Laplacian, 205 launches), plus
# FETCH_SIZE / WRITE_SIZE passes (the 16.8 MB working set is Infinity-Cache resident: the counters
# show fabric traffic, not HBM).  Usage on the GPU box: bash scripts/profile_config2.sh <tag>
set -u
TAG=${1:-r02}
OUT=$PWD/gpurun_out/prof_c2_$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
for pass in "trace:--kernel-trace --stats" "fetch:--pmc FETCH_SIZE" "write:--pmc WRITE_SIZE"; do
  name=${pass%%:*}; args=${pass#*:}
  timeout -k 10 300 rocprofv3 $args -d "$OUT/$name" -o "$name" --output-format csv -- \
      python3 scripts/config2_kernel.py > "$OUT/$name.log" 2>&1
  rc=$?; echo "=== $name rc=$rc"; grep '^{' "$OUT/$name.log" || tail -3 "$OUT/$name.log"
  [ $rc -ne 0 ] && exit $rc
done
exit 0
