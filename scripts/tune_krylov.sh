#!/bin/bash
# A/B the Krylov kernel grids (env overrides read by krylov.hip) on the full bench.
for cfg in "2048 1073741824" "8192 1073741824" "1024 1073741824" "4096 4096"; do
  set -- $cfg
  echo "== MDOT_BLOCKS=$1 COMBO_BLOCKS=$2"
  NKHIP_MDOT_BLOCKS=$1 NKHIP_COMBO_BLOCKS=$2 timeout -k 10 300 python bench.py --steps 4 --warmup 1 --cpu-baseline off | python -c "
import json,sys; d=json.loads(sys.stdin.readlines()[-1]); k=d['kernels']
print('steps/s', d['value'], 'ms/step', d['ms_per_step'], {n:(v['ms'],v['GB/s']) for n,v in k.items() if n in ('krylov_mdot','krylov_combo','reduce_final','sh_fdjvp')})" || exit $?
done
