#!/bin/bash
# rocprofv3 --kernel-trace --stats over the bench for environment variants (one box):
#   bash scripts/stats_ab.sh "name:ENV=V ..." ...  -> gpurun_out/stats_<name>/
mkdir -p gpurun_out
export TMPDIR=/tmp
for spec in "$@"; do
  name=${spec%%:*}; envs=${spec#*:}
  for kv in $envs; do export "$kv"; done
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/stats_$name -o s --output-format csv -- \
      python3 bench.py --steps 3 --warmup 2 --cpu-baseline off --extra off > gpurun_out/stats_$name.log 2>&1
  rc=$?; echo "=== $name rc=$rc"; [ $rc -ne 0 ] && exit $rc
  for kv in $envs; do unset "${kv%%=*}"; done
done
exit 0
