#!/bin/bash
# Round 6: the ALT instantiations taken for short bands only -- the march-direction tests, the
# round-5 fused kernel against this one on 512 .. 4096 rows (one call), the N = 8 rank's slab
# machinery at world size one for each slab path (pushed, pushed + tail, edge + halo, in-kernel
# exchange), and the one-GPU per-step chain (host loop / device control / device control in the
# fused launch's tail) on the driver's window.
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
O=$PWD/gpurun_out/r06h
mkdir -p "$O"
L=$PWD/iterative-solvers-summer-2020_amd/nkhip
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread \
    tests/test_gpu_fused.py -k "march_direction" > "$O/tests.log" 2>&1 || { tail -30 "$O/tests.log"; exit 1; }
tail -1 "$O/tests.log"
for rep in 1 2; do
  for v in r05 r06; do
    if [ $v = r05 ]; then env="NKHIP_LIB=$L/libnkhip_r05.so"; else env="NKHIP_BENCH_DUMMY=1"; fi
    echo "$v $(env $env timeout -k 10 200 python3 scripts/slab_size_probe.py 512 1024 2048 4096 2>/dev/null | tr '\n' ' ')" | tee -a "$O/ab.log"
  done
done
for v in pushed pushed_tail edge_halo in_kernel; do
  case $v in
    pushed) env="NKHIP_SLAB_PUSH=1" ;;
    pushed_tail) env="NKHIP_ARN_TAIL=1" ;;
    edge_halo) env="NKHIP_SLAB_PUSH=0" ;;
    in_kernel) env="NKHIP_SLAB_XK=2" ;;
  esac
  echo "$v $(env $env timeout -k 10 300 python3 scripts/slab_peer_probe.py 512 4096 2>/dev/null | tr '\n' ' ')" | tee -a "$O/slabpeer.log"
done
bash scripts/gpu_r06g.sh && cp gpurun_out/r06g_chain.log "$O/chain.log"
