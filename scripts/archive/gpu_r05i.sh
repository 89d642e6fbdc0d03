#!/bin/bash
# Round 5: isolated fused A/B (this tree vs the committed arnoldi.hip (r5a) vs round 4 (base)),
# config 2's tile kernel with the lane exchange (parity tests + rocprof durations), and a bench
# A/B of the combinations' own edge arrays (NKHIP_COMBO_EDGES).
set -u
TAG=${1:-r05i}
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
NKHIP_TILE_XCH=1 timeout -k 10 300 python3 -u -m pytest tests -m gpu -x -q -k "config2 or tile or lap5 or operator" --timeout 200 --timeout-method thread > gpurun_out/${TAG}_xch_tests.log 2>&1 || { tail -20 gpurun_out/${TAG}_xch_tests.log; exit 1; }
tail -1 gpurun_out/${TAG}_xch_tests.log
for rep in 1 2; do
for v in "2 0" "2 1" "4 1"; do
  set -- $v
  d=gpurun_out/${TAG}_c2_$1_$2_$rep
  NKHIP_TILE_ROWS=$1 NKHIP_TILE_XCH=$2 timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $d -o c2 --output-format csv -- python3 scripts/config2_kernel.py > $d.log 2>&1 || { tail $d.log; exit 1; }
  python3 - $d "$1 $2" <<'PY'
import csv, glob, sys
for f in glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "tile" in r["Name"] or "march" in r["Name"]:
            print("rows/xch", sys.argv[2], r["Calls"], round(float(r["AverageNs"]) / 1e3, 3), "us",
                  round(float(r["MinNs"]) / 1e3, 3), round(float(r["MaxNs"]) / 1e3, 3))
PY
done
done
timeout -k 10 600 bash scripts/arn_ab.sh 4,8,12,16,18,19,20,22,24,28,33,35 A r5a base > gpurun_out/${TAG}_ab.log 2>&1; rc=$?
cat gpurun_out/${TAG}_ab.log
[ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
  for v in 1 0; do
    NKHIP_COMBO_EDGES=$v timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --cpu-baseline off --extra off --pmc off > gpurun_out/${TAG}_w20_$v.log 2>&1 || { tail -c 1500 gpurun_out/${TAG}_w20_$v.log; exit 1; }
    python3 -c "
import json; d=json.loads([l for l in open('gpurun_out/${TAG}_w20_$v.log') if l.startswith('{')][-1])
print('combo_edges=$v', d['value'], d['ms_per_arnoldi_step'], d['roofline']['frac'], d['kernels'].get('krylov_combo',{}).get('avg_us'), d['kernels'].get('edge_gather',{}).get('launches'))"
  done
done
