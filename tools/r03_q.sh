#!/bin/bash
# forward kernel: parity, phase clocks, bench leg
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r03_${1:-q}
mkdir -p $OUT
cd $R
T="python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu -p no:cacheprovider"
timeout -k 10 400 $T tests/test_gpu_forward.py -k "stream or full_size" > $OUT/tests_fwd.log 2>&1 || { echo "forward tests failed"; tail -60 $OUT/tests_fwd.log; exit 12; }
tail -1 $OUT/tests_fwd.log
timeout -k 10 200 python3 tools/fwd_phase.py active rand > $OUT/phase.log 2>&1 || { echo "phase failed"; tail -20 $OUT/phase.log; exit 13; }
cat $OUT/phase.log
timeout -k 10 200 python3 bench.py --config c5 --variants active,rand --no-cpu-baseline --no-e2e --no-others --steps 10 --warmup 3 > $OUT/bench_c5fwd.log 2>&1 || { echo "bench c5 failed"; tail -20 $OUT/bench_c5fwd.log; exit 14; }
python3 -c "
import json; d=json.loads([l for l in open('$OUT/bench_c5fwd.log') if l.startswith('{')][-1])
print('c5', d['value'], d['roofline']['frac'], 'fwd', d.get('forward'))"
