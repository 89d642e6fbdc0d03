#!/bin/bash
# SQ counters of the fused Arnoldi kernel (scripts/arnoldi_bench.py), one rocprofv3 pass per
# counter set.  Usage on the GPU box: bash scripts/pmc_arnoldi.sh <tag>   (ARN_NVS selects nv)
set -u
TAG=${1:-arn}
OUT=$PWD/gpurun_out/pmc_$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp ARN_NVS=${ARN_NVS:-8,24}
pass() {  # pass <name> <counters...>
  local name=$1; shift
  echo "=== $name ($(date +%T))"
  timeout -s KILL 120 rocprofv3 --pmc "$@" -d "$OUT/$name" -o "$name" --output-format csv -- \
      python3 scripts/arnoldi_bench.py > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"
  if [ $rc -ne 0 ]; then tail -n 5 "$OUT/$name.log"; exit $rc; fi
}
pass sq1 SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS
pass sq2 SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VALU
python3 - "$OUT" <<'PY'
import collections, csv, glob, sys
agg = collections.defaultdict(lambda: collections.defaultdict(float))
cnt = collections.defaultdict(int)
for f in glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("nk::(anonymous namespace)::", "")
        agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
        cnt[(k, r["Counter_Name"])] += 1
for k, d in sorted(agg.items()):
    if "arnoldi" not in k:
        continue
    n = max(cnt[(k, c)] for c in d)
    print(k, "dispatches", n)
    print("   " + "  ".join(f"{c}={v / cnt[(k, c)]:.4g}" for c, v in sorted(d.items())))
PY
