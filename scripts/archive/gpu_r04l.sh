#!/bin/bash
# Where a step's idle GPU time goes: kernel traces of the default bench with the host-loop and
# the device-side Arnoldi control on one GPU, and of the world-of-one slab path.
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
ARGS="--steps 4 --warmup 1 --extra off --cpu-baseline off --pmc off --probes off"
for v in "host:NKHIP_DEVCTL=0:" "devctl:NKHIP_DEVCTL=1:" "slab::--peer-self"; do
  name=${v%%:*}; rest=${v#*:}; envs=${rest%%:*}; extra=${rest#*:}
  rm -rf gpurun_out/gap_$name
  env $envs timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/gap_$name -o k --output-format csv -- \
    python3 bench.py $ARGS $extra > gpurun_out/gap_$name.log 2>&1 || { echo "$name failed"; tail -5 gpurun_out/gap_$name.log; exit 1; }
  echo "=== $name"; python3 scripts/gap_analysis.py gpurun_out/gap_$name 12
done
