#!/bin/bash
# Same-box A/B of env-selected variants on the full bench (per-Arnoldi-step time is comparable
# across step counts).  Usage: bash scripts/ab_bench.sh "ENV=.. ENV2=.." "ENV=.." ...
for cfg in "$@"; do
  echo "== $cfg"
  env $cfg timeout -k 10 300 python bench.py --steps 4 --warmup 1 --cpu-baseline off --extra off --pmc off | python -c "
import json,sys; d=json.loads(sys.stdin.readlines()[-1]); k=d['kernels']
print('steps/s', d['value'], 'ms/step', d['ms_per_step'], 'ms/arnoldi', d['ms_per_arnoldi_step'], {n:(v['avg_us'],v['GB/s']) for n,v in k.items() if n in ('krylov_mdot','krylov_combo','reduce_final','sh_fdjvp')})" || exit $?
done
