#!/bin/bash
# Round 6, after the write-through pushes and the fence-free control launch: every slab path of
# the N = 8 rank's machinery at world size one (512 / 4096 rows), and the plain slab beside it.
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=$PWD/gpurun_out/r06q
mkdir -p "$O"
timeout -k 10 200 python3 scripts/slab_size_probe.py 512 4096 > "$O/slabsize.log" 2>&1 || { tail -20 "$O/slabsize.log"; exit 1; }
for rep in 1 2; do
for v in pushed pushed_tail edge_halo in_kernel; do
  case $v in
    pushed) env="NKHIP_SLAB_PUSH=1" ;;
    pushed_tail) env="NKHIP_ARN_TAIL=1" ;;
    edge_halo) env="NKHIP_SLAB_PUSH=0" ;;
    in_kernel) env="NKHIP_SLAB_XK=2" ;;
  esac
  env $env timeout -k 10 300 python3 scripts/slab_peer_probe.py 512 4096 > "$O/p_${v}_$rep.log" 2>&1 \
      || { echo "probe $v failed: $?"; tail -20 "$O/p_${v}_$rep.log"; exit 1; }
  echo "$v $rep $(grep '{' "$O/p_${v}_$rep.log" | tr '\n' ' ')" >> "$O/slabpeer.log"
done
done
echo done
