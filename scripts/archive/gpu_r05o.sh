#!/bin/bash
# Round 5: droplet / PMA2 kernels -- tests, PMA stage timing, config 3 / PMA2 steps/s, kernel
# durations (rocprofv3 over scripts/config3_ab.py).
set -u
TAG=${1:-r05o}
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_droplet.py tests/test_gpu_mems.py -x -q --timeout 300 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1 || { tail -30 gpurun_out/${TAG}_tests.log; exit 1; }
tail -1 gpurun_out/${TAG}_tests.log
NKHIP_PMA_TIMING=1 timeout -k 10 200 python3 scripts/config3_ab.py > gpurun_out/${TAG}_pmatime.log 2>&1 || { tail -20 gpurun_out/${TAG}_pmatime.log; exit 1; }
grep "pma us" gpurun_out/${TAG}_pmatime.log | sort | uniq -c | sort -rn | head -2
for rep in 1 2; do timeout -k 10 200 python3 scripts/config3_ab.py 2>&1 | tail -1; done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_prof -o c3 --output-format csv -- python3 scripts/config3_ab.py > gpurun_out/${TAG}_prof.log 2>&1 || { tail -20 gpurun_out/${TAG}_prof.log; exit 1; }
python3 - gpurun_out/${TAG}_prof <<'PY'
import csv, glob, sys
for f in glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True):
    for r in list(csv.DictReader(open(f)))[:8]:
        print(r["Name"][:60], r["Calls"], round(float(r["TotalDurationNs"]) / 1e6, 2), "ms", round(float(r["AverageNs"]) / 1e3, 2), "us")
PY
