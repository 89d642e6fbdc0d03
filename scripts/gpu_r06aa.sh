#!/bin/bash
# Round 6: the control launches reduce with the control's loads issued after the partial loads
# (reduce_column_ctl): the control-launch stage probe, the whole GPU suite, the A/B against the
# previous build (r06x) on the world-of-one slab (pushed path).
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=$PWD/gpurun_out/${1:-r06s}
mkdir -p "$O"
L=$PWD/iterative-solvers-summer-2020_amd/nkhip
NKHIP_LIB=$L/libnkhip_cprobe.so timeout -k 10 200 python3 scripts/dbg/ctl_probe.py 512 > "$O/ctl512.log" 2>&1 || { tail -20 "$O/ctl512.log"; exit 1; }
grep -v "Warn\|Gloo\|amdgpu.ids\|socket" "$O/ctl512.log"
timeout -k 10 1500 python -u -m pytest -x -q -m gpu --timeout 300 --timeout-method thread tests \
    > "$O/gputest.log" 2>&1 || { tail -30 "$O/gputest.log"; exit 1; }
tail -1 "$O/gputest.log"
for rep in 1 2; do
  for v in prev new; do
    if [ $v = prev ]; then env="NKHIP_LIB=$L/libnkhip_prev.so"; else env="NKHIP_BENCH_DUMMY=1"; fi
    env $env timeout -k 10 300 python3 scripts/slab_peer_probe.py 512 4096 > "$O/p_${v}_$rep.log" 2>&1 \
        || { echo "probe $v $rep failed: $?"; tail -20 "$O/p_${v}_$rep.log"; exit 1; }
    echo "$v $rep $(tr '\n' ' ' < "$O/p_${v}_$rep.log")" >> "$O/ab.log"
  done
done
echo "ab done"
