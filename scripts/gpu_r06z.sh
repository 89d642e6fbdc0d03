#!/bin/bash
# Round 6: the one-GPU chain under the host loop and under device control, as the device sees it
# (rocprofv3 kernel trace: kernel durations and the idle gaps between consecutive kernels), the
# driver's window.
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=$PWD/gpurun_out/${1:-r06z}
mkdir -p "$O"
for v in host devctl; do
  if [ $v = host ]; then export NKHIP_DEVCTL=0; else export NKHIP_DEVCTL=1; fi
  timeout -k 10 600 rocprofv3 --kernel-trace -d "$O/$v" -o "$v" --output-format csv -- python3 bench.py --steps 20 --warmup 5 --cpu-baseline off --extra off --pmc off --probes off > "$O/$v.log" 2>&1 || { echo "$v failed"; tail -20 "$O/$v.log"; exit 1; }
  f=$(find "$O/$v" -name "*kernel_trace.csv" | head -1)
  echo "== $v $(grep '^{' "$O/$v.log" | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_arnoldi_step"])')"
  python3 scripts/dbg/gap_trace.py "$f" | tee "$O/${v}_gaps.txt"
done
