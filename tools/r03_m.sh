#!/bin/bash
# SQ counters on both streaming kernels (tools/sq_stream.sh), then C5 with
# plain vs nontemporal output stores in the streaming kernel
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r03_${1:-m}
mkdir -p $OUT
cd $R
bash tools/sq_stream.sh r03_${1:-m}/sq || exit 10
for M in 1 0; do
  TDBG_STREAM_STORE=$M timeout -k 10 120 python3 bench.py --config c5 --no-cpu-baseline --no-e2e --no-forward --no-others --steps 20 --warmup 5 > $OUT/c5_store$M.log 2>&1 || { echo "bench store $M failed"; tail -20 $OUT/c5_store$M.log; exit 11; }
  python3 -c "
import json; d=json.loads([l for l in open('$OUT/c5_store$M.log') if l.startswith('{')][-1])
print('store $M', {v: (x['GiBps'], x['roofline_frac'], x['kernel_ms']) for v, x in d['config']['variants'].items()})"
done
