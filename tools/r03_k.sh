#!/bin/bash
# the driver's default bench command, timed
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r03_${1:-k}
mkdir -p $OUT
cd $R
S=$(date +%s)
timeout -k 10 600 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench.log 2>&1 || { echo "bench failed"; tail -30 $OUT/bench.log; exit 11; }
echo "bench took $(( $(date +%s) - S )) s"
grep '^{' $OUT/bench.log > $OUT/bench.json
python3 -c "
import json; d=json.load(open('$OUT/bench.json'))
print('value', d['value'], d['config']['variant'], 'frac', d['roofline']['frac'])
for v,x in d['config']['variants'].items(): print(' ', v, x['GiBps'], x['roofline_frac'], x['kernel_ms'])
for c,o in d['config'].get('other_configs',{}).items(): print(c, o['value_GiBps'], o['roofline']['frac'], o.get('cpu_baseline',{}).get('value'))
print('100k', d['config'].get('c5_100k_single_gpu'))
print('e2e', d['config'].get('e2e_GiBps')); print('fwd', d.get('forward',{}).get('value'), d.get('forward',{}).get('roofline_frac')); print('cpu', d.get('cpu_baseline'))
"
