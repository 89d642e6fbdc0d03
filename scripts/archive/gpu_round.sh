#!/bin/bash
# One GPU-box session: tests, smoke, short bench.  Stops at the first step that ends in anything
# other than success / ordinary test failure (fault, abort, timeout).
mkdir -p gpurun_out
step() {  # step <name> <timeout-seconds> <cmd...>
  local name=$1 t=$2; shift 2
  echo "=== $name ($(date +%T))"
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"; tail -n 25 "gpurun_out/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
  return 0
}
for s in "$@"; do
  case $s in
    tests)  step pytest_gpu 900 python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread ;;
    alltests) step pytest_gpu 900 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread ;;
    smoke)  step smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
    bench)  step bench 900 python bench.py --steps 5 --warmup 1 --cpu-baseline off --extra off ;;
    benchfull) step bench_full 900 python bench.py ;;
  esac
done
