#!/bin/bash
# Round measurements: devctl accounting check (plain vs device control), rocprofv3 profile of the
# default-window bench (scripts/profile.sh), then the driver's default bench line.
set -o pipefail
mkdir -p gpurun_out
for v in "plain:" "plain_devctl:NKHIP_DEVCTL=1" "rccl:--rccl-self"; do
  name=${v%%:*}; rest=${v#*:}; args=""; envs=""
  for t in $rest; do case $t in *=*) envs="$envs $t";; *) args="$args $t";; esac; done
  out=$(env $envs MASTER_ADDR=127.0.0.1 MASTER_PORT=$((29600 + RANDOM % 200)) timeout -k 10 300 \
        python bench.py --steps 5 --warmup 1 --cpu-baseline off --extra off $args 2>/dev/null | grep '^{') || exit $?
  echo "$name $(echo "$out" | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); k=d['kernels']; print(d['value'], d['ms_per_arnoldi_step'], d['roofline']['frac'], k['arnoldi_fused']['launches'], k['arnoldi_fused']['avg_us'])")"
done
bash scripts/profile.sh ${PROF_TAG:-r02d} || exit $?
timeout -k 10 900 python bench.py > gpurun_out/bench_default.log 2>&1; rc=$?; tail -c 3000 gpurun_out/bench_default.log; exit $rc
