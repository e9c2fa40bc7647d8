#!/bin/bash
# forward kernel (parity, phases, bench leg) + C1 shuffle kernel (tests, bench)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r03_${1:-r}
mkdir -p $OUT
cd $R
T="python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu -p no:cacheprovider"
timeout -k 10 400 $T tests/test_gpu_forward.py -k "stream or full_size or config" > $OUT/tests_fwd.log 2>&1 || { echo "forward tests failed"; tail -60 $OUT/tests_fwd.log; exit 12; }
tail -1 $OUT/tests_fwd.log
timeout -k 10 400 $T tests/test_gpu_stream_small.py > $OUT/tests_small.log 2>&1 || { echo "small tests failed"; tail -60 $OUT/tests_small.log; exit 13; }
tail -1 $OUT/tests_small.log
timeout -k 10 200 python3 tools/fwd_phase.py active rand > $OUT/phase.log 2>&1 || { echo "phase failed"; tail -20 $OUT/phase.log; exit 14; }
grep -v amdgpu.ids $OUT/phase.log
timeout -k 10 120 python3 bench.py --config c1 --no-cpu-baseline --no-e2e --no-forward --steps 20 --warmup 5 > $OUT/bench_c1.log 2>&1 || { echo "bench c1 failed"; tail -20 $OUT/bench_c1.log; exit 15; }
python3 -c "
import json; d=json.loads([l for l in open('$OUT/bench_c1.log') if l.startswith('{')][-1])
print('c1', d['value'], d['roofline']['frac'], d['roofline']['kernel_ms'], d['config'].get('stream_tiles_timed'))"
timeout -k 10 200 python3 bench.py --config c5 --variants active,rand --no-cpu-baseline --no-e2e --no-others --steps 10 --warmup 3 > $OUT/bench_c5fwd.log 2>&1 || { echo "bench c5 failed"; tail -20 $OUT/bench_c5fwd.log; exit 16; }
python3 -c "
import json; d=json.loads([l for l in open('$OUT/bench_c5fwd.log') if l.startswith('{')][-1])
print('c5', d['value'], d['roofline']['frac'], 'fwd', d.get('forward',{}).get('value'), d.get('forward',{}).get('roofline_frac'))"
