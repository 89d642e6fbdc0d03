#!/bin/bash
# A/B of two builds of the C-ABI on the default bench, alternating inside one gpurun call (the
# box-to-box spread is larger than most effects): bash scripts/ab_lib.sh <libA> <libB> [rounds]
# [bench args...].  Prints steps/s, the dominant-kernel and JVP fractions and the box's copy rate.
set -u
A=$1; B=$2; R=${3:-2}; shift 3 || shift $#
ARGS=${*:-"--steps 10 --warmup 2 --extra off --cpu-baseline off --pmc off"}
mkdir -p gpurun_out
for i in $(seq 1 "$R"); do
  for L in "$A" "$B"; do
    tag=$(basename "$L" .so)_$i
    NKHIP_LIB=$PWD/$L timeout -k 10 300 python3 bench.py $ARGS > gpurun_out/ab_$tag.log 2>&1 || { echo "$tag failed"; exit 1; }
    python3 - "$tag" gpurun_out/ab_$tag.log <<'PY'
import json, sys
d = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
r, j = d["roofline"], d["jvp_roofline"]
print(f"{sys.argv[1]:24s} steps/s {d['value']:.3f} ms/arn {d['ms_per_arnoldi_step']:.4f} "
      f"{r['kernel']} {r['frac']:.4f} jvp {j['frac']:.4f} ({j['avg_us']:.1f} us) "
      f"copy {d['copy_bandwidth']['GB/s']:.0f} GB/s (torch {d['copy_bandwidth']['torch_copy_GB/s']:.0f})")
PY
  done
done
