#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/pmcnt
LIB=$PWD/iterative-solvers-summer-2020_amd/nkhip/libnkhip_b24.so
for nt in 1 0; do
  NKHIP_ARN_NT=$nt NKHIP_LIB=$LIB ARN_NVS=24 timeout -k 10 120 python -u scripts/arnoldi_bench.py 2>/dev/null | grep '^{' | sed "s/^/nt=$nt /" || exit $?
  for c in FETCH_SIZE WRITE_SIZE; do
    NKHIP_ARN_NT=$nt NKHIP_LIB=$LIB ARN_NVS=24 timeout -s KILL 120 rocprofv3 --pmc $c -d gpurun_out/pmcnt/nt${nt}_$c -o p --output-format csv -- python3 scripts/arnoldi_bench.py > gpurun_out/pmcnt/nt${nt}_$c.log 2>&1 || exit $?
  done
done
