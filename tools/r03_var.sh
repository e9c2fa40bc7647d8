#!/bin/bash
# A/B timing of prebuilt engine variants (varlibs/lib*.so) on C5 active
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r03_${1:-var}
mkdir -p $OUT
cd $R
for v in H B A H A; do
  cp varlibs/lib$v.so tiledb_amd/libtiledb_amd.so
  timeout -k 10 200 python3 bench.py --config c5 --variants active --no-cpu-baseline --no-e2e --no-others --no-forward --steps 20 --warmup 5 > $OUT/bench_$v.log 2>&1 || { echo "bench $v failed"; tail -20 $OUT/bench_$v.log; exit 16; }
  python3 -c "
import json; d=json.loads([l for l in open('$OUT/bench_$v.log') if l.startswith('{')][-1])
print('$v', {k: (v['GiBps'], v['roofline_frac'], v['kernel_ms']) for k, v in d['config']['variants'].items()})"
done
