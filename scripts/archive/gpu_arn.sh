# Fused Arnoldi kernel: tests, then microbench configurations (one process each: the tuning
# knobs are read once per process).  Usage: bash scripts/gpu_arn.sh [tests] [bench] [tune]
set -o pipefail
mkdir -p gpurun_out
for step in "$@"; do
case $step in
tests)
  timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_fused.py > gpurun_out/fused.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -5 gpurun_out/fused.log
  if [ $rc -gt 1 ]; then exit $rc; fi ;;
bench)
  ARN_TAG=default timeout -k 10 120 python -u scripts/arnoldi_bench.py > gpurun_out/arn_default.log 2>&1 || exit $? ;;
tune)
  for pf in ${ARN_PFS:-1 2 3 4 6}; do
    NKHIP_LIB=$PWD/iterative-solvers-summer-2020_amd/nkhip/libnkhip_tune.so NKHIP_ARN_PF=$pf ARN_TAG=pf$pf \
      timeout -k 10 120 python -u scripts/arnoldi_bench.py > gpurun_out/arn_pf$pf.log 2>&1 || exit $?
  done ;;
esac
done
echo done
