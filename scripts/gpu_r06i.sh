#!/bin/bash
# Round 6 state: the whole GPU suite, smoke(), rocprofv3 passes over the default one-GPU bench
# (kernel trace + stats, FETCH_SIZE, WRITE_SIZE), the default bench line and the driver's window
# (steps 6-25), the short-slab probe and the N = 8 rank's slab machinery at world size one.
set -u
TAG=${1:-r06i}
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
L=$PWD/iterative-solvers-summer-2020_amd/nkhip
timeout -k 10 1000 python3 -u -m pytest tests -m gpu -x -q --timeout 900 --timeout-method thread \
  > gpurun_out/${TAG}_gputest.log 2>&1
rc=$?
tail -5 gpurun_out/${TAG}_gputest.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/${TAG}_smoke.log 2>&1 || { tail -5 gpurun_out/${TAG}_smoke.log; exit 1; }
tail -1 gpurun_out/${TAG}_smoke.log
bash scripts/profile.sh $TAG > gpurun_out/${TAG}_prof.log 2>&1 || { tail -20 gpurun_out/${TAG}_prof.log; exit 1; }
tail -3 gpurun_out/${TAG}_prof.log
timeout -k 10 900 python3 bench.py > gpurun_out/${TAG}_bench.log 2>&1 || { tail -c 1500 gpurun_out/${TAG}_bench.log; exit 1; }
tail -c 400 gpurun_out/${TAG}_bench.log
timeout -k 10 600 python3 bench.py --steps 20 --warmup 5 --cpu-baseline off --extra off > gpurun_out/${TAG}_bench_w20.log 2>&1 || { tail -c 1500 gpurun_out/${TAG}_bench_w20.log; exit 1; }
python3 -c "
import json; d=json.loads([l for l in open('gpurun_out/${TAG}_bench_w20.log') if l.startswith('{')][-1])
print('window 6-25:', d['value'], d['ms_per_arnoldi_step'], d['roofline']['frac'], d['jvp_roofline']['frac'])"
timeout -k 10 300 python3 scripts/slab_size_probe.py 512 1024 2048 4096 > gpurun_out/${TAG}_slabsize.log 2>&1 && grep "{" gpurun_out/${TAG}_slabsize.log
# the N = 8 rank's slab machinery at world size one (pushed path), 512 and 4096 rows
timeout -k 10 300 python3 scripts/slab_peer_probe.py 512 4096 > gpurun_out/${TAG}_slabpeer.log 2>&1 && grep "{" gpurun_out/${TAG}_slabpeer.log
