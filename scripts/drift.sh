#!/bin/bash
# Run-to-run spread of the default bench on one box: N separate processes back to back (each
# allocates its own workspace pool), with the placement-probe times of each run.
N=${1:-6}
for i in $(seq 1 "$N"); do
  timeout -k 10 300 python3 bench.py --steps 10 --warmup 2 --extra off --cpu-baseline off > gpurun_out/drift_$i.log 2>&1 || exit 1
  python3 -c "
import json;d=json.loads(open('gpurun_out/drift_$i.log').read().strip().splitlines()[-1]);r=d['roofline']
print('run $i', d['value'], r['frac'], d['jvp_roofline']['frac'], 'probe', [round(x) for x in d.get('pool_probe_us', [])])"
done
