#!/bin/bash
# Round 6: does the device control win on one GPU once the fused pass's outputs are written
# through (ARN_OUT_POL=16: no dirty-L2 write-back for the next pass to run into)?  Host loop /
# device control x plain / write-through outputs on the driver's window, and the world-of-one
# pushed slab (device control) with both libraries, alternating in one call.
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=$PWD/gpurun_out/${1:-r06w}
mkdir -p "$O"
L=$PWD/iterative-solvers-summer-2020_amd/nkhip
for rep in 1 2; do
  for v in host devctl host_op16 devctl_op16; do
    case $v in
      host) env="NKHIP_DEVCTL=0" ;;
      devctl) env="NKHIP_DEVCTL=1" ;;
      host_op16) env="NKHIP_DEVCTL=0 NKHIP_LIB=$L/libnkhip_op16.so" ;;
      devctl_op16) env="NKHIP_DEVCTL=1 NKHIP_LIB=$L/libnkhip_op16.so" ;;
    esac
    line=$(env $env timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --cpu-baseline off \
        --extra off --pmc off --probes off 2>/dev/null | grep "^{") || { echo "$v failed"; exit 1; }
    python3 -c "
import json,sys; d=json.loads(sys.argv[1]); k=d['kernels']
print('$v', d['value'], d['ms_per_arnoldi_step'], d['roofline']['frac'], {c: (v['launches'], v['avg_us']) for c, v in k.items() if c in ('arnoldi_fused','reduce_final','arnoldi_ctl')})" "$line" >> "$O/chain.log"
  done
done
for v in plain op16; do
  if [ $v = op16 ]; then env="NKHIP_LIB=$L/libnkhip_op16.so"; else env="NKHIP_BENCH_DUMMY=1"; fi
  env $env timeout -k 10 300 python3 scripts/slab_peer_probe.py 512 4096 > "$O/p_$v.log" 2>&1 \
      || { echo "probe $v failed: $?"; tail -20 "$O/p_$v.log"; exit 1; }
  echo "$v $(grep '{' "$O/p_$v.log" | tr '\n' ' ')" >> "$O/slab.log"
done
cat "$O/chain.log"
