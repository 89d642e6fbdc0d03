#!/bin/bash
# Round 5: config 2's tile kernel variants (rows per thread, store policy), kernel-only durations.
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
for rep in 1 2; do
for v in "1 0" "2 0" "4 0" "1 1" "2 1" "4 1"; do
  set -- $v
  d=gpurun_out/r05f_c2_$1_$2_$rep
  NKHIP_TILE_ROWS=$1 NKHIP_TILE_NT=$2 timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $d -o c2 --output-format csv -- python3 scripts/config2_kernel.py > $d.log 2>&1 || { tail $d.log; exit 1; }
  python3 - $d "$1 $2" <<'PY'
import csv, glob, sys
for f in glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "tile" in r["Name"] or "march" in r["Name"]:
            print("rows/nt", sys.argv[2], r["Calls"], round(float(r["AverageNs"]) / 1e3, 3), "us",
                  round(float(r["MinNs"]) / 1e3, 3), round(float(r["MaxNs"]) / 1e3, 3))
PY
done
done
NKHIP_TILE_MAX=0 timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/r05f_march -o c2 --output-format csv -- python3 scripts/config2_kernel.py > gpurun_out/r05f_march.log 2>&1 || exit 1
python3 - gpurun_out/r05f_march march <<'PY'
import csv, glob, sys
for f in glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "tile" in r["Name"] or "march" in r["Name"]:
            print(sys.argv[2], r["Calls"], round(float(r["AverageNs"]) / 1e3, 3), "us")
PY
