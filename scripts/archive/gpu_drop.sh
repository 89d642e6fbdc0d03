#!/bin/bash
# Droplet (config 3) step breakdown: per-step wall time, then rocprofv3 kernel stats + trace.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 120 python3 scripts/droplet_run.py 5 > gpurun_out/drop_run.log 2>&1 || exit $?
tail -n 3 gpurun_out/drop_run.log
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d gpurun_out/drop_prof -o drop --output-format csv -- \
  python3 scripts/droplet_run.py 3 > gpurun_out/drop_prof.log 2>&1 || exit $?
head -12 gpurun_out/drop_prof/drop_kernel_stats.csv
