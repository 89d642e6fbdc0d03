#!/bin/bash
# Round 6: the build with write-through pushes (KMAX back at 2) and the fence-free control launch:
# every-basis-length kernel test and the edges cases first, then the whole GPU suite, then the
# A/B against the r06i library on the world-of-one slab.
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=$PWD/gpurun_out/r06p
mkdir -p "$O"
L=$PWD/iterative-solvers-summer-2020_amd/nkhip
timeout -k 10 120 python3 scripts/dbg/edges_diff.py r06p > "$O/edges.log" 2>&1 || { tail -20 "$O/edges.log"; exit 1; }
timeout -k 10 1500 python -u -m pytest -x -q -m gpu --timeout 300 --timeout-method thread tests \
    > "$O/gputest.log" 2>&1 || { tail -30 "$O/gputest.log"; exit 1; }
tail -1 "$O/gputest.log"
for rep in 1 2; do
  for v in r06i new; do
    if [ $v = r06i ]; then env="NKHIP_LIB=$L/libnkhip_r06i.so"; else env="NKHIP_BENCH_DUMMY=1"; fi
    env $env timeout -k 10 300 python3 scripts/slab_peer_probe.py 512 4096 > "$O/p_${v}_$rep.log" 2>&1 \
        || { echo "probe $v $rep failed: $?"; tail -20 "$O/p_${v}_$rep.log"; exit 1; }
    echo "$v $rep $(tr '\n' ' ' < "$O/p_${v}_$rep.log")" >> "$O/ab.log"
  done
done
echo "ab done"
