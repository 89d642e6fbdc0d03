#!/bin/bash
# A/B stencil variants (env knobs read by stencil.hip) on the FD-JVP / SH13 microbench at 4096^2.
# usage: bash scripts/ab_stencil.sh "NKHIP_PF=1" "NKHIP_PF=2 NKHIP_RY_MAX=16" ...
export KB_ONLY=${KB_ONLY:-sh_fdjvp,sh13,torch_copy}
for cfg in "$@"; do
  echo "== $cfg"
  env $cfg timeout -k 10 120 python scripts/kernel_bench.py ${KB_SIZES:-4096} || exit $?
done
