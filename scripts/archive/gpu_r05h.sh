#!/bin/bash
# Round 5: the wide layout's 32-bit row arithmetic / pinned scalars and the combinations' own
# edge arrays -- bounds-checked solve, the GPU suite, isolated fused A/B (this tree vs the
# committed arnoldi.hip (r5a) vs round 4 (base)), and a bench A/B of NKHIP_COMBO_EDGES.
set -u
TAG=${1:-r05h}
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
for g in "256 256" "128 512"; do
  timeout -k 10 120 python3 -u scripts/dbg/bounds_probe.py $g > gpurun_out/${TAG}_bounds.log 2>&1 || { tail -5 gpurun_out/${TAG}_bounds.log; exit 1; }
  tail -2 gpurun_out/${TAG}_bounds.log
done
timeout -k 10 1000 python3 -u -m pytest tests -m gpu -x -q --timeout 900 --timeout-method thread \
  > gpurun_out/${TAG}_gputest.log 2>&1
rc=$?
tail -5 gpurun_out/${TAG}_gputest.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 bash scripts/arn_ab.sh 4,8,12,16,18,19,20,22,24,28,33,34,35 A r5a base > gpurun_out/${TAG}_ab.log 2>&1 || { cat gpurun_out/${TAG}_ab.log; exit 1; }
cat gpurun_out/${TAG}_ab.log
for rep in 1 2; do
  for v in 1 0; do
    NKHIP_COMBO_EDGES=$v timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --cpu-baseline off --extra off --pmc off > gpurun_out/${TAG}_w20_$v.log 2>&1 || { tail -c 1500 gpurun_out/${TAG}_w20_$v.log; exit 1; }
    python3 -c "
import json; d=json.loads([l for l in open('gpurun_out/${TAG}_w20_$v.log') if l.startswith('{')][-1])
print('combo_edges=$v', d['value'], d['ms_per_arnoldi_step'], d['roofline']['frac'], d['kernels'].get('krylov_combo',{}).get('avg_us'), d['kernels'].get('edge_gather',{}).get('launches'))"
  done
done
