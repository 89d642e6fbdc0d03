#!/bin/bash
# Round-end measurements: rocprofv3 profile (scripts/profile.sh), then the default bench.
set -o pipefail
mkdir -p gpurun_out
bash scripts/profile.sh ${PROF_TAG:-r02f} || exit $?
timeout -k 10 900 python bench.py > gpurun_out/bench_default.log 2>&1; rc=$?
grep '^{' gpurun_out/bench_default.log | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_arnoldi_step'], d['roofline']['frac'], d['per_step'], d['other_configs']['config3']['gpu_steps_per_s'])"
exit $rc
