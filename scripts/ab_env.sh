#!/bin/bash
# A/B of runtime switches on the default bench, alternating inside one gpurun call:
#   bash scripts/ab_env.sh <rounds> "<env settings A>" "<env settings B>" ...
# e.g. bash scripts/ab_env.sh 2 "NKHIP_PF=1" "NKHIP_PF=2".  BENCH_ARGS overrides the bench args.
set -u
R=$1; shift
ARGS=${BENCH_ARGS:-"--steps 10 --warmup 2 --extra off --cpu-baseline off --pmc off"}
mkdir -p gpurun_out
for i in $(seq 1 "$R"); do
  k=0
  for E in "$@"; do
    k=$((k + 1))
    tag="v${k}_$i"
    env $E timeout -k 10 300 python3 bench.py $ARGS > gpurun_out/abe_$tag.log 2>&1 || { echo "$E failed"; exit 1; }
    python3 - "$E" gpurun_out/abe_$tag.log <<'PY'
import json, sys
d = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
r, j = d["roofline"], d["jvp_roofline"]
ks = d["kernels"]
extra = " ".join(f"{k}:{v['avg_us']:.0f}us" for k, v in ks.items() if k in ("sh_trial", "sh_bold"))
print(f"{sys.argv[1]:40s} steps/s {d['value']:.3f} ms/arn {d['ms_per_arnoldi_step']:.4f} "
      f"{r['kernel']} {r['frac']:.4f} jvp {j['frac']:.4f} ({j['avg_us']:.1f} us) {extra} "
      f"copy {d['copy_bandwidth']['GB/s']:.0f}")
PY
  done
done
