#!/bin/bash
# Round 5 final tree: the GPU suite and smoke() (no bench: r05u measured the same sources).
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 1000 python3 -u -m pytest tests -m gpu -x -q --timeout 900 --timeout-method thread > gpurun_out/r05x_gputest.log 2>&1
rc=$?
tail -3 gpurun_out/r05x_gputest.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r05x_smoke.log 2>&1 || { tail -5 gpurun_out/r05x_smoke.log; exit 1; }
tail -1 gpurun_out/r05x_smoke.log
