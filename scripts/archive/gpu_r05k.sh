#!/bin/bash
# Round 5: droplet stencil stages in column strips -- droplet / PMA2 tests, PMA stage timing,
# config 3 / PMA2 steps/s.
set -u
TAG=${1:-r05k}
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_droplet.py tests/test_gpu_mems.py -x -q --timeout 300 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1 || { tail -30 gpurun_out/${TAG}_tests.log; exit 1; }
tail -1 gpurun_out/${TAG}_tests.log
NKHIP_PMA_TIMING=1 timeout -k 10 200 python3 scripts/config3_ab.py > gpurun_out/${TAG}_pmatime.log 2>&1 || { tail -20 gpurun_out/${TAG}_pmatime.log; exit 1; }
grep "pma us" gpurun_out/${TAG}_pmatime.log | sort | uniq -c | sort -rn | head -3
for rep in 1 2; do timeout -k 10 200 python3 scripts/config3_ab.py 2>&1 | tail -1; done
