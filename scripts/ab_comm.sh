#!/bin/bash
# World-size-1 cost of the slab path: plain periodic slab vs the peer-memory communicator vs
# RCCL (bench.py --peer-self / --rccl-self), alternating inside one gpurun call (VARIANTS=...).
#   bash scripts/ab_comm.sh [rounds]
set -u
R=${1:-2}
ARGS="--steps 10 --warmup 2 --extra off --cpu-baseline off --pmc off"
mkdir -p gpurun_out
for i in $(seq 1 "$R"); do
  for V in ${VARIANTS:-plain peer peer0 rccl}; do
    F=1; XK=0; PUSH=1; TAIL=0
    case $V in
      plain) X="" ;;
      peer) X="--peer-self" ;;  # pushed halo rows (default): no exchange before the fused pass
      peert) X="--peer-self"; TAIL=1 ;;  # reduction + all-reduce + control in the fused launch's tail
      peerex) X="--peer-self"; PUSH=0 ;;  # the slab edge + halo exchange kernel before it
      peer0) X="--peer-self"; F=0 ;;  # separate communicator launches (NKHIP_PEER_FUSE=0)
      peerxk) X="--peer-self"; XK=2 ;;  # the fused kernel's edge bands exchange (NKHIP_SLAB_XK)
      rccl) X="--rccl-self" ;;
    esac
    NKHIP_ARN_TAIL=$TAIL NKHIP_SLAB_PUSH=$PUSH NKHIP_SLAB_XK=$XK NKHIP_PEER_FUSE=$F timeout -k 10 300 python3 bench.py $ARGS $X > gpurun_out/abc_${V}_$i.log 2>&1 || { echo "$V failed"; tail -5 gpurun_out/abc_${V}_$i.log; exit 1; }
    python3 - "$V" gpurun_out/abc_${V}_$i.log <<'PY'
import json, sys
d = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
k = d["kernels"]
parts = " ".join(f"{n}:{v['avg_us']:.1f}us" for n, v in k.items()
                 if n in ("halo", "halo_push", "reduce_final", "arnoldi_ctl", "arnoldi_edge",
                          "arnoldi_fused"))
print(f"{sys.argv[1]:6s} steps/s {d['value']:.3f} ms/arn {d['ms_per_arnoldi_step']:.4f} "
      f"fused {d['roofline']['frac']:.4f} {parts}")
PY
  done
done
