#!/bin/bash
# small-image streaming kernel: its GPU tests, then C3a/C3b/C4 bench lines
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r03_${1:-n}
mkdir -p $OUT
cd $R
timeout -k 10 400 python3 -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_stream_small.py -p no:cacheprovider > $OUT/tests.log 2>&1 \
  || { echo "tests failed"; tail -60 $OUT/tests.log; exit 10; }
tail -3 $OUT/tests.log
for C in c3a c3b c4; do
  timeout -k 10 120 python3 bench.py --config $C --no-cpu-baseline --no-e2e --no-forward --steps 20 --warmup 5 > $OUT/bench_$C.log 2>&1 || { echo "bench $C failed"; tail -20 $OUT/bench_$C.log; exit 11; }
  python3 -c "
import json; d=json.loads([l for l in open('$OUT/bench_$C.log') if l.startswith('{')][-1])
print('$C', d['value'], d['roofline']['frac'], d['roofline']['kernel_ms'], d['config'].get('stream_tiles_timed'), d['config'].get('fallback_tiles_timed'))"
done
