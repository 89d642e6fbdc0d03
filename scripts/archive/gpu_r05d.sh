#!/bin/bash
# Round 5: 32-bit row math + register-resident grid scalars in the pair kernel, and the
# speculative first JVP of each LGMRES call -- parity (fused/NK tests), then isolated kernel A/B
# against the round-4 library (libnkhip_base.so) and bench A/B (incl. device control on one GPU).
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
L=$PWD/iterative-solvers-summer-2020_amd/nkhip
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_fused.py tests/test_gpu_nk.py -m gpu -x -q \
  --timeout 300 --timeout-method thread > gpurun_out/r05d_tests.log 2>&1 || { tail -30 gpurun_out/r05d_tests.log; exit 1; }
tail -3 gpurun_out/r05d_tests.log
timeout -k 10 500 bash scripts/arn_ab.sh 4,8,12,16,18,19,20,21,22,24,28,35 A base > gpurun_out/r05d_ab.log 2>&1 || { tail gpurun_out/r05d_ab.log; exit 1; }
cat gpurun_out/r05d_ab.log
BENCH_STEPS=10 timeout -k 10 900 bash scripts/bench_ab.sh "new:" "base:NKHIP_LIB=$L/libnkhip_base.so" "nospec:NKHIP_SPEC_JVP=0" "devctl:NKHIP_DEVCTL=1" > gpurun_out/r05d_bench.log 2>&1 || { tail gpurun_out/r05d_bench.log; exit 1; }
cat gpurun_out/r05d_bench.log
