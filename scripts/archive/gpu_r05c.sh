#!/bin/bash
# Round 5: the vector-pair layout's short end (nv 19-22) -- mailbox statistics per launch
# (libnkhip_mbstat.so), SQ counters of the fused kernel at nv 18/19/20/24/35 (product library),
# and the timing with every consumer recomputing (NKHIP_ARN_MBOX=2) beside the default.
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
L=$PWD/iterative-solvers-summer-2020_amd/nkhip
NKHIP_LIB=$L/libnkhip_mbstat.so ARN_MBSTAT=1 ARN_NVS=19,20,21,22,24,28,35 timeout -k 10 200 \
  python3 -u scripts/arnoldi_bench.py > gpurun_out/r05c_mbstat.log 2>&1 || { tail gpurun_out/r05c_mbstat.log; exit 1; }
cat gpurun_out/r05c_mbstat.log
timeout -k 10 400 bash scripts/arn_ab.sh 18,19,20,21,22,24,35 A A:NKHIP_ARN_MBOX=2 > gpurun_out/r05c_ab.log 2>&1 || { tail gpurun_out/r05c_ab.log; exit 1; }
cat gpurun_out/r05c_ab.log
ARN_NVS=18,19,20,24,35 timeout -k 10 600 bash scripts/pmc_arnoldi.sh r05c > gpurun_out/r05c_pmc.log 2>&1 || { tail gpurun_out/r05c_pmc.log; exit 1; }
cat gpurun_out/r05c_pmc.log
