# Microbenchmark libnkhip variants (NKHIP_LIB) of the fused Arnoldi kernel, one process each.
# Usage on the GPU box: bash scripts/arn_variants.sh A B C ...  (A = the default library)
set -o pipefail
mkdir -p gpurun_out
export ARN_NVS=${ARN_NVS:-1,4,8,16,24,32}
for v in "$@"; do
  lib=$PWD/iterative-solvers-summer-2020_amd/nkhip/libnkhip_$v.so
  [ "$v" = A ] && lib=$PWD/iterative-solvers-summer-2020_amd/nkhip/libnkhip.so
  echo "== $v"
  NKHIP_LIB=$lib timeout -k 10 120 python -u scripts/arnoldi_bench.py > gpurun_out/arnv_$v.log 2>&1 || exit $?
  grep -v amdgpu.ids gpurun_out/arnv_$v.log | python3 -c "import sys,json; r=[json.loads(l) for l in sys.stdin]; print(' '.join(('E' if x['ext'] else 'n')+str(x['nv'])+':'+str(int(x['us'])) for x in r))"
done
