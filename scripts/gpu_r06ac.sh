#!/bin/bash
# Round 6: the final combination's batch (NKHIP_COMBO_UNR: basis vectors whose loads are in
# flight together, 2 / 4 / 8) on the driver's window, alternating in one call.
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=$PWD/gpurun_out/${1:-r06ac}
mkdir -p "$O"
for rep in 1 2; do
  for u in 2 4 8; do
    line=$(NKHIP_COMBO_UNR=$u timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --cpu-baseline off --extra off --pmc off --probes off 2>/dev/null | grep "^{") || { echo "unr $u failed"; exit 1; }
    python3 -c "
import json,sys; d=json.loads(sys.argv[1]); k=d['kernels']
print('unr $u', d['value'], d['ms_per_arnoldi_step'], k['krylov_combo']['avg_us'], k['krylov_combo']['GB/s'], k['arnoldi_fused']['avg_us'])" "$line" >> "$O/ab.log"
  done
done
cat "$O/ab.log"
