#!/bin/bash
# Round-3 GPU pass c: streaming-kernel tests (coded + raw DD), the C5 bench
# line with all three variants, and kernel traces of rand/ramp/active.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r03_${1:-c}
mkdir -p $OUT
export TMPDIR=/tmp
cd $R
timeout -k 10 400 python -u -m pytest tests/test_gpu_stream.py -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/pytest_stream.log 2>&1 || { echo "pytest failed"; grep -E "PASS|FAIL|Error|error|assert" $OUT/pytest_stream.log | head -60; tail -30 $OUT/pytest_stream.log; exit 11; }
tail -3 $OUT/pytest_stream.log
timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-e2e --no-forward > $OUT/bench.log 2>&1 || { echo "bench failed"; tail -30 $OUT/bench.log; exit 12; }
grep '^{' $OUT/bench.log | grep -o '"variants": {.*}}, "min' | head -1
for V in rand ramp active; do
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace_$V -o run -- python3 $R/bench.py --config c5 --variants $V --no-cpu-baseline --no-e2e --no-forward --steps 10 --warmup 2 > $OUT/trace_$V.log 2>&1 || { echo "trace $V failed"; tail -20 $OUT/trace_$V.log; exit 13; }
  echo "== $V"; grep -h "unfilter\|fixup" $OUT/trace_$V/*kernel_stats.csv | cut -c1-150
done
echo done
