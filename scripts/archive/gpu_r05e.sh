#!/bin/bash
# Round 5: tile kernel (config 2), speculative JVP with a polled trial reduction, sc1 output
# stores of the fused kernel (A/B), the 8-process tail stall probe.
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
L=$PWD/iterative-solvers-summer-2020_amd/nkhip
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_ops.py tests/test_gpu_fused.py tests/test_gpu_nk.py \
  -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r05e_tests.log 2>&1 || { tail -30 gpurun_out/r05e_tests.log; exit 1; }
tail -2 gpurun_out/r05e_tests.log
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/r05e_c2 -o c2 --output-format csv -- python3 scripts/config2_kernel.py > gpurun_out/r05e_c2.log 2>&1 || { tail gpurun_out/r05e_c2.log; exit 1; }
python3 - <<'PY'
import csv, glob
for f in glob.glob("gpurun_out/r05e_c2/**/*kernel_stats.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        print("config2", r["Name"][:60], r["Calls"], float(r["AverageNs"]) / 1e3, "us")
PY
BENCH_STEPS=10 timeout -k 10 900 bash scripts/bench_ab.sh "new:" "sc1:NKHIP_LIB=$L/libnkhip_sc1.so" "nospec:NKHIP_SPEC_JVP=0" > gpurun_out/r05e_bench.log 2>&1 || { tail gpurun_out/r05e_bench.log; exit 1; }
cat gpurun_out/r05e_bench.log
for v in spec nospec; do
  e=""; [ $v = nospec ] && e="NKHIP_SPEC_JVP=0"
  env $e timeout -k 10 400 python3 bench.py --steps 10 --warmup 2 --cpu-baseline off --extra off > gpurun_out/r05e_full_$v.log 2>&1 || { tail gpurun_out/r05e_full_$v.log; exit 1; }
  python3 -c "
import json,sys; d=json.loads([l for l in open('gpurun_out/r05e_full_$v.log') if l.startswith('{')][-1])
j=d['jvp_roofline']; print('$v', d['value'], d['ms_per_arnoldi_step'], 'fused', d['roofline']['frac'], 'jvp', j['frac'], j.get('avg_us'), j.get('event_avg_us'), 'traffic', d['traffic_measurement'].get('classes',{}).get('sh_fdjvp'), 'copy', d['copy_bandwidth']['GB/s'])"
done
for P in 4 8; do
  timeout -k 10 200 python3 scripts/dbg/tail8_probe.py $P 256 > gpurun_out/r05e_tail$P.log 2>&1 || { tail gpurun_out/r05e_tail$P.log; exit 1; }
  cat gpurun_out/r05e_tail$P.log
done
