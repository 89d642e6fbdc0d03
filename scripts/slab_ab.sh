#!/bin/bash
# Slab-path timing on one GPU: bench.py through the RCCL communicator at world size 1 (self halo,
# in-stream all-reduces) with and without the interior/halo overlap, beside the plain single slab.
set -o pipefail
mkdir -p gpurun_out
for rep in 1 2; do
  for v in "plain:" "rccl_serial:--rccl-self" "rccl_overlap:--rccl-self NKHIP_SLAB_OVERLAP=1" "rccl_ov16:--rccl-self NKHIP_SLAB_OVERLAP=1 NKHIP_SLAB_RESERVE_CUS=16"; do
    name=${v%%:*}; rest=${v#*:}; args=""; envs=""
    for t in $rest; do case $t in *=*) envs="$envs $t";; *) args="$args $t";; esac; done
    out=$(env $envs MASTER_ADDR=127.0.0.1 MASTER_PORT=$((29600 + RANDOM % 200)) timeout -k 10 300 \
          python bench.py --steps 10 --warmup 2 --cpu-baseline off --extra off $args 2>/dev/null | grep '^{') || exit $?
    echo "$rep $name $(echo "$out" | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); k=d['kernels']; print(d['value'], d['ms_per_arnoldi_step'], {n: (v['launches'], v['avg_us']) for n, v in k.items() if n.startswith('arnoldi') or n in ('halo','reduce_final')})")"
  done
done
