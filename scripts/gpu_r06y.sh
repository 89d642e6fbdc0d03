#!/bin/bash
# Round 6: the one-GPU headline with the round-state fused kernels (r06i sources, linked with the
# current rest) against this build, alternating in one call: the driver's window (steps 6-25) and
# the default bench window, fused pass and step rate.
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=$PWD/gpurun_out/${1:-r06y}
mkdir -p "$O"
L=$PWD/iterative-solvers-summer-2020_amd/nkhip
for rep in 1 2; do
  for v in r06i new; do
    if [ $v = r06i ]; then env="NKHIP_LIB=$L/libnkhip_r06iarn.so"; else env="NKHIP_BENCH_DUMMY=1"; fi
    for w in w20 default; do
      if [ $w = w20 ]; then args="--steps 20 --warmup 5"; else args=""; fi
      line=$(env $env timeout -k 10 300 python3 bench.py $args --cpu-baseline off --extra off --pmc off --probes off 2>/dev/null | grep "^{") || { echo "$v $w failed"; exit 1; }
      python3 -c "
import json,sys; d=json.loads(sys.argv[1]); k=d['kernels']
print('$v $w', d['value'], d['ms_per_arnoldi_step'], d['roofline']['frac'], k['arnoldi_fused']['avg_us'])" "$line" >> "$O/ab.log"
    done
  done
done
cat "$O/ab.log"
