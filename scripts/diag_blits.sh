#!/bin/bash
# Which runtime API calls issue the __amd_rocclr_* blits of the world-of-one peer slab path:
# rocprofv3 kernel + HIP API trace (no counters) over a short --peer-self bench run, then the
# API stats and the blits' correlated API calls.
#   bash scripts/diag_blits.sh [extra bench args]
set -eu
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/diag_blits
rm -rf "$OUT"; mkdir -p "$OUT"
timeout -k 10 240 rocprofv3 --kernel-trace --hip-trace --stats --output-format csv -d "$OUT" -o run -- \
  python3 bench.py --peer-self --steps 2 --warmup 1 --extra off --cpu-baseline off --pmc off --probes off "$@" \
  > "$OUT/bench.log" 2>&1
python3 scripts/blit_origin.py "$OUT" | tee "$OUT/origin.txt"
