#!/bin/bash
# Round 6: the slab halo-row prologue in one round of slot loads (KMAX covering a block's
# 2 (BW + 4) points) against the r06i library, on the N = 8 rank's slab machinery at world size
# one (pushed path), 512 and 4096 rows, two alternations in one call; then the fused-kernel tests
# that run slab paths.
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
O=$PWD/gpurun_out/${1:-r06j}
mkdir -p "$O"
L=$PWD/iterative-solvers-summer-2020_amd/nkhip
for rep in 1 2; do
  for v in r06i new; do
    if [ $v = r06i ]; then env="NKHIP_LIB=$L/libnkhip_r06i.so"; else env="NKHIP_BENCH_DUMMY=1"; fi
    env $env timeout -k 10 300 python3 scripts/slab_peer_probe.py 512 4096 > "$O/p_${v}_$rep.log" 2>&1 \
        || { echo "probe $v $rep failed: $?"; tail -20 "$O/p_${v}_$rep.log"; exit 1; }
    echo "$v $rep $(tr '\n' ' ' < "$O/p_${v}_$rep.log")" | tee -a "$O/ab.log"
  done
done
timeout -k 10 900 python -u -m pytest -x -q --timeout 600 --timeout-method thread \
    tests/test_gpu_peer.py tests/test_gpu_fused.py -k "slab or peer" > "$O/tests.log" 2>&1 || { tail -30 "$O/tests.log"; exit 1; }
tail -1 "$O/tests.log"
