#!/bin/bash
# Round 5: config 3's time split -- PMA per-stage timing and a kernel trace of five droplet steps.
set -u
TAG=${1:-r05j}
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
NKHIP_PMA_TIMING=1 timeout -k 10 200 python3 scripts/config3_ab.py > gpurun_out/${TAG}_pmatime.log 2>&1 || { tail -20 gpurun_out/${TAG}_pmatime.log; exit 1; }
sort gpurun_out/${TAG}_pmatime.log | uniq -c | sort -rn | head -8
tail -2 gpurun_out/${TAG}_pmatime.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_prof -o c3 --output-format csv -- python3 scripts/config3_ab.py > gpurun_out/${TAG}_prof.log 2>&1 || { tail -20 gpurun_out/${TAG}_prof.log; exit 1; }
python3 - gpurun_out/${TAG}_prof <<'PY'
import csv, glob, sys
for f in glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True):
    rows = list(csv.DictReader(open(f)))
    for r in rows[:14]:
        print(r["Name"][:70], r["Calls"], round(float(r["TotalDurationNs"]) / 1e6, 2), "ms", round(float(r["AverageNs"]) / 1e3, 2), "us")
PY
