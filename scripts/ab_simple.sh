for cfg in "$@"; do
  echo "== $cfg"
  env $cfg timeout -k 10 300 python bench.py --steps 4 --warmup 1 --cpu-baseline off --extra off --pmc off | python -c "
import json,sys; d=json.loads(sys.stdin.readlines()[-1]); print('steps/s', d['value'], 'ms/arnoldi', d['ms_per_arnoldi_step'], 'frac', d['kernel_time_frac_of_wall'])" || exit $?
done
