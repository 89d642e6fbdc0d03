#!/bin/bash
# test_fused_kernel_edges_identical[True-40-130] failed on the r06m build: every case of it, on the
# r06i library and on this one, outputs kept for a cross-comparison.
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=$PWD/gpurun_out/r06n
mkdir -p "$O"
L=$PWD/iterative-solvers-summer-2020_amd/nkhip
NKHIP_LIB=$L/libnkhip_r06i.so timeout -k 10 120 python3 scripts/dbg/edges_diff.py r06i > "$O/r06i.log" 2>&1 || { tail -20 "$O/r06i.log"; exit 1; }
timeout -k 10 120 python3 scripts/dbg/edges_diff.py new > "$O/new.log" 2>&1 || { tail -20 "$O/new.log"; exit 1; }
timeout -k 10 120 python3 scripts/dbg/edges_diff.py new2 > "$O/new2.log" 2>&1 || { tail -20 "$O/new2.log"; exit 1; }
grep EDGES "$O/r06i.log" "$O/new.log" "$O/new2.log" | cut -c1-400
