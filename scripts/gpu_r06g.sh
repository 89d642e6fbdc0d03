#!/bin/bash
# Round 6: the one-GPU per-Arnoldi-step chain (verdict item 6): the driver's window (steps 6-25)
# with the host loop (default), the device-side control (NKHIP_DEVCTL=1: reduction + control
# launch, no host round trip) and the device-side control in the fused launch's tail
# (NKHIP_DEVCTL=1 NKHIP_ARN_TAIL=1), alternating in one call.
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
O=gpurun_out/${1:-r06g}_chain.log
for rep in 1 2; do
  for v in host devctl tail; do
    case $v in
      host) env="NKHIP_DEVCTL=0" ;;
      devctl) env="NKHIP_DEVCTL=1" ;;
      tail) env="NKHIP_DEVCTL=1 NKHIP_ARN_TAIL=1" ;;
    esac
    line=$(env $env timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --cpu-baseline off \
        --extra off --pmc off --probes off 2>/dev/null | grep "^{") || { echo "$v failed"; exit 1; }
    python3 -c "
import json,sys; d=json.loads(sys.argv[1]); k=d['kernels']
print('$v', d['value'], d['ms_per_arnoldi_step'], d['roofline']['frac'], {c: (v['launches'], v['avg_us']) for c, v in k.items() if c in ('arnoldi_fused','reduce_final','arnoldi_ctl')})" "$line" | tee -a $O
  done
done
