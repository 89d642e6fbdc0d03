#!/bin/bash
# Round 6: fence-free control launch (sc1 hand-off, the tail's form) on top of the write-through
# pushed rows: A/B against the r06i library on the N = 8 rank's slab machinery at world size one
# (512 and 4096 rows, two alternations), then the whole GPU suite.
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=$PWD/gpurun_out/${1:-r06m}
mkdir -p "$O"
L=$PWD/iterative-solvers-summer-2020_amd/nkhip
for rep in 1 2; do
  for v in r06i new; do
    if [ $v = r06i ]; then env="NKHIP_LIB=$L/libnkhip_r06i.so"; else env="NKHIP_BENCH_DUMMY=1"; fi
    env $env timeout -k 10 300 python3 scripts/slab_peer_probe.py 512 4096 > "$O/p_${v}_$rep.log" 2>&1 \
        || { echo "probe $v $rep failed: $?"; tail -20 "$O/p_${v}_$rep.log"; exit 1; }
    echo "$v $rep $(tr '\n' ' ' < "$O/p_${v}_$rep.log")" >> "$O/ab.log"
  done
done
echo "ab done"
timeout -k 10 1500 python -u -m pytest -x -q -m gpu --timeout 300 --timeout-method thread tests \
    > "$O/gputest.log" 2>&1 || { tail -30 "$O/gputest.log"; exit 1; }
tail -1 "$O/gputest.log"
