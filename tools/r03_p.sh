#!/bin/bash
# new kernels: small-image stream tests, bitshuffle + forward parity, then
# C2/C2i/C3a/C3b/C4 lines and the C5 forward leg
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r03_${1:-p}
mkdir -p $OUT
cd $R
T="python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu -p no:cacheprovider"
timeout -k 10 400 $T tests/test_gpu_stream_small.py > $OUT/tests_small.log 2>&1 || { echo "small tests failed"; tail -60 $OUT/tests_small.log; exit 10; }
tail -1 $OUT/tests_small.log
timeout -k 10 400 $T tests/test_gpu_forward.py -k "stream or full_size or config" > $OUT/tests_fwd.log 2>&1 || { echo "forward tests failed"; tail -60 $OUT/tests_fwd.log; exit 12; }
tail -1 $OUT/tests_fwd.log
timeout -k 10 400 $T tests/test_gpu_parity.py -k "C2 or spec or bitshuffle" > $OUT/tests_bit.log 2>&1 || { echo "bitshuffle tests failed"; tail -60 $OUT/tests_bit.log; exit 13; }
tail -1 $OUT/tests_bit.log
for C in c2 c2i c3a c3b c4; do
  timeout -k 10 120 python3 bench.py --config $C --no-cpu-baseline --no-e2e --no-forward --steps 20 --warmup 5 > $OUT/bench_$C.log 2>&1 || { echo "bench $C failed"; tail -20 $OUT/bench_$C.log; exit 11; }
  python3 -c "
import json; d=json.loads([l for l in open('$OUT/bench_$C.log') if l.startswith('{')][-1])
print('$C', d['value'], d['roofline']['frac'], d['roofline']['kernel_ms'], d['config'].get('stream_tiles_timed'), d['config'].get('fallback_tiles_timed'))"
done
timeout -k 10 200 python3 bench.py --config c5 --variants active,rand --no-cpu-baseline --no-e2e --no-others --steps 10 --warmup 3 > $OUT/bench_c5fwd.log 2>&1 || { echo "bench c5 failed"; tail -20 $OUT/bench_c5fwd.log; exit 14; }
python3 -c "
import json; d=json.loads([l for l in open('$OUT/bench_c5fwd.log') if l.startswith('{')][-1])
print('c5', d['value'], d['roofline']['frac'], 'fwd', d.get('forward'))"
