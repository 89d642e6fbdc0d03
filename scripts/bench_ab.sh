#!/bin/bash
# A/B of environment switches on the headline bench (alternating runs, one box):
#   bash scripts/bench_ab.sh "name:ENV=V ENV2=V2" "name2:" ...   (BENCH_ARGS: extra bench.py flags)
set -o pipefail
mkdir -p gpurun_out
for rep in 1 2; do
  for spec in "$@"; do
    name=${spec%%:*}; envs=${spec#*:}
    out=$(env $envs timeout -k 10 300 python bench.py --steps ${BENCH_STEPS:-10} --warmup 2 --cpu-baseline off --extra off ${BENCH_ARGS:-} 2>/dev/null | grep '^{') || exit $?
    echo "$rep $name $(echo "$out" | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_arnoldi_step'], d['roofline']['frac'], d['kernel_time_frac_of_wall'])")"
  done
done
