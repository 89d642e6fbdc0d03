#!/bin/bash
# Why is the fused kernel faster on the RCCL slab path?  bench A/B with host vs device control
# on the plain slab, then rocprofv3 kernel stats of plain vs rccl-self.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for rep in 1 2; do
  for v in "plain:" "plain_devctl:NKHIP_DEVCTL=1" "rccl:--rccl-self" "rccl_hostctl:--rccl-self NKHIP_DEVCTL=0"; do
    name=${v%%:*}; rest=${v#*:}; args=""; envs=""
    for t in $rest; do case $t in *=*) envs="$envs $t";; *) args="$args $t";; esac; done
    out=$(env $envs MASTER_ADDR=127.0.0.1 MASTER_PORT=$((29600 + RANDOM % 200)) timeout -k 10 300 \
          python bench.py --steps 5 --warmup 1 --cpu-baseline off --extra off $args 2>/dev/null | grep '^{') || exit $?
    echo "$rep $name $(echo "$out" | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); k=d['kernels']; print(d['value'], d['ms_per_arnoldi_step'], d['roofline']['frac'], k['arnoldi_fused']['avg_us'], d['per_step'])")"
  done
done
for v in plain rccl; do
  args=""; [ $v = rccl ] && args="--rccl-self"
  MASTER_ADDR=127.0.0.1 MASTER_PORT=29711 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/why_$v -o why --output-format csv -- \
    python3 bench.py --steps 3 --warmup 1 --cpu-baseline off --extra off $args > gpurun_out/why_$v.log 2>&1 || exit $?
done
