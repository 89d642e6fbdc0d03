#!/bin/bash
# rocprofv3 passes over the bench (kernel trace + stats, then HBM counters in separate passes),
# each with the solver's launch log for the per-dispatch traffic match (scripts/traffic_match.py).
# Usage on the GPU box: bash scripts/profile.sh <tag> [bench args...]
set -u
TAG=${1:-r02}; shift || true
ARGS=${*:-"--steps 3 --warmup 1 --cpu-baseline off --extra off --pmc off"}
OUT=$PWD/gpurun_out/prof_$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
run() {  # run <name> <timeout> <rocprof args...>
  local name=$1 t=$2; shift 2
  echo "=== $name ($(date +%T))"
  NKHIP_LAUNCH_LOG="$OUT/$name.launches" timeout -k 10 "$t" rocprofv3 "$@" -d "$OUT/$name" \
      -o "$name" --output-format csv -- python3 bench.py $ARGS > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"; tail -n 3 "$OUT/$name.log"
  if [ $rc -ne 0 ]; then echo "stopping after $name"; exit $rc; fi
}
run trace 600 --kernel-trace --stats
run fetch 600 --pmc FETCH_SIZE
run write 600 --pmc WRITE_SIZE
# the three runs are the same deterministic program: their launch logs must agree
cmp -s "$OUT/trace.launches" "$OUT/fetch.launches" && cmp -s "$OUT/trace.launches" "$OUT/write.launches" \
  && echo "launch logs identical" || echo "WARNING: launch logs differ between passes"
python3 scripts/traffic_match.py "$TAG" "$OUT" "$OUT/trace.launches" > "$OUT/traffic_match.log" 2>&1
cp profiles/${TAG}_traffic.json "$OUT/" 2>/dev/null || true
echo "traffic_match rc=$?"
find "$OUT" -name "*.csv" | head -20
