#!/bin/bash
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_droplet.py tests/test_gpu_mems.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r05s_tests.log 2>&1; rc=$?
tail -3 gpurun_out/r05s_tests.log
[ $rc -eq 0 ] || exit $rc
for m in plain numpy pytest conftest npz; do timeout -k 10 120 python3 scripts/dbg/drop_create_probe.py $m 2>&1 | grep create; done
