#!/bin/bash
# Band height of the march kernels (FD-JVP in situ): for each NKHIP_BLOCKS target, the default
# bench (in-situ jvp_roofline) and a profile.sh pass (per-dispatch traffic), one gpurun call.
#   bash scripts/jvp_sweep.sh 4096 2048 1536 ...
set -u
mkdir -p gpurun_out
for B in "$@"; do
  NKHIP_BLOCKS=$B bash scripts/ab_env.sh 1 "NKHIP_BLOCKS=$B" || exit 1
  NKHIP_BLOCKS=$B bash scripts/profile.sh jvp_b$B > gpurun_out/prof_jvp_b$B.log 2>&1 || exit 1
  grep -A12 '"sh_fdjvp"' gpurun_out/prof_jvp_b$B/traffic_match.log | grep -E 'traffic_over_alg|avg_us' | tr '\n' ' '; echo " <- B=$B"
done
