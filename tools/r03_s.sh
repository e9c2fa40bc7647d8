#!/bin/bash
# C5 coded kernel change: stream parity tests, then the C5 bench (all variants)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r03_${1:-s}
mkdir -p $OUT
cd $R
T="python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu -p no:cacheprovider"
timeout -k 10 400 $T tests/test_gpu_stream.py > $OUT/tests_stream.log 2>&1 || { echo "stream tests failed"; tail -60 $OUT/tests_stream.log; exit 12; }
tail -1 $OUT/tests_stream.log
timeout -k 10 500 $T tests/test_gpu_parity.py > $OUT/tests_parity.log 2>&1 || { echo "parity tests failed"; tail -60 $OUT/tests_parity.log; exit 13; }
tail -1 $OUT/tests_parity.log
timeout -k 10 240 python3 bench.py --config c5 --no-cpu-baseline --no-e2e --no-others --no-forward --steps 20 --warmup 5 > $OUT/bench_c5.log 2>&1 || { echo "bench c5 failed"; tail -20 $OUT/bench_c5.log; exit 16; }
python3 -c "
import json; d=json.loads([l for l in open('$OUT/bench_c5.log') if l.startswith('{')][-1])
print('c5', d['value'], {k: (v['GiBps'], v['roofline_frac'], v['kernel_ms']) for k, v in d['config']['variants'].items()})"
