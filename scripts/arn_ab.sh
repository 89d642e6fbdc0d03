#!/bin/bash
# A/B of fused-Arnoldi library variants at one basis length, alternating runs (box noise):
#   bash scripts/arn_ab.sh <nvs> <variant[:ENV=VAL]>...   e.g.  arn_ab.sh 24 b24 nodot24 tune24:NKHIP_ARN_PF=2
set -o pipefail
mkdir -p gpurun_out
nvs=$1; shift
for rep in 1 2; do
  for spec in "$@"; do
    v=${spec%%:*}; envs=""; [ "$spec" != "$v" ] && envs=${spec#*:}
    lib=$PWD/iterative-solvers-summer-2020_amd/nkhip/libnkhip_$v.so
    [ "$v" = A ] && lib=$PWD/iterative-solvers-summer-2020_amd/nkhip/libnkhip.so
    res=$(env $envs NKHIP_LIB=$lib ARN_NVS=$nvs timeout -k 10 120 python -u scripts/arnoldi_bench.py 2>/dev/null | grep '^{' | python3 -c "import sys,json; r=[json.loads(l) for l in sys.stdin]; print(' '.join(('E' if x['ext'] else 'n')+str(x['nv'])+':'+str(int(x['us']))+'us/'+str(x['frac']) for x in r))") || exit $?
    echo "$rep $spec  $res"
  done
done
