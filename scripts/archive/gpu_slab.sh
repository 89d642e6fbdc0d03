#!/bin/bash
# Full -m gpu suite, then the slab path's cost at world size 1 (RCCL self-halo) beside the plain
# single slab, alternating runs.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread \
  > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -4 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
  for v in "plain:" "rccl:--rccl-self"; do
    name=${v%%:*}; args=${v#*:}
    out=$(MASTER_ADDR=127.0.0.1 MASTER_PORT=$((29600 + RANDOM % 200)) timeout -k 10 300 \
          python bench.py --steps 10 --warmup 2 --cpu-baseline off --extra off $args 2>/dev/null | grep '^{') || exit $?
    echo "$rep $name $(echo "$out" | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); k=d['kernels']; print(d['value'], d['ms_per_arnoldi_step'], d['roofline']['frac'], {n: (v['launches'], v['avg_us']) for n, v in k.items() if n.startswith('arnoldi') or n in ('halo','reduce_final')})")"
  done
done
