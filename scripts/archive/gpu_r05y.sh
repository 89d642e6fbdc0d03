#!/bin/bash
# Round 5: the N > 1 bench line end to end on one GPU (two ranks sharing device 0): 4096^2
# headline on 2 row slabs, comm self-tests, slab A/B and config 5's 16384^2 leg.  A rehearsal of
# the driver's SCALE run (the ranks share one GPU's bandwidth: not a scaling number).
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
NKHIP_BENCH_ONE_DEVICE=1 timeout -k 10 900 python3 bench.py --gpus 2 --steps 3 --warmup 1 > gpurun_out/r05y_bench_n2.log 2>&1; rc=$?
tail -c 3000 gpurun_out/r05y_bench_n2.log
exit $rc
