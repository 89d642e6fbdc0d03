#!/bin/bash
# Bisect of the EXT fused kernel's wrong w' on the r06m build: nv-7-only libraries (r06i sources;
# current; current with a plain push store; current with 2 slot items per thread; both), every
# test_fused_kernel_edges_identical case against a torch FD reference.
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=$PWD/gpurun_out/r06o
mkdir -p "$O"
L=$PWD/iterative-solvers-summer-2020_amd/nkhip
for v in r06i base plain k2 pk2; do
  NKHIP_LIB=$L/libnkhip_dbg_$v.so timeout -k 10 120 python3 scripts/dbg/edges_diff.py dbg_$v > "$O/$v.log" 2>&1 || { tail -20 "$O/$v.log"; exit 1; }
  echo "== $v"; grep EDGES "$O/$v.log" | python3 -c "
import sys,json
for l in sys.stdin:
    d=json.loads(l.split('EDGES ',1)[1]); print(d['ext'],d['ny'],d['nx'],'%.1e %.1e'%(d['w1_err'],d['w2_err']))"
done
