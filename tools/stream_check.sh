#!/bin/bash
# Streaming C5 kernel iteration: its parity tests, the C5-related parity
# cases, then a short C5 bench.  Each GPU step time-limited, chained.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/stream_${1:-x}
mkdir -p $OUT
cd $R
timeout -k 10 300 python -u -m pytest tests/test_gpu_c5tile.py -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/pytest_stream.log 2>&1 || { echo "stream tests failed"; tail -40 $OUT/pytest_stream.log; exit 11; }
tail -3 $OUT/pytest_stream.log
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "c5 or C5 or spec19 or spec20" > $OUT/pytest_c5.log 2>&1 || { echo "c5 parity failed"; tail -40 $OUT/pytest_c5.log; exit 12; }
tail -2 $OUT/pytest_c5.log
timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-e2e ${BENCH_ARGS} > $OUT/bench.log 2>&1 || { echo "bench failed"; tail -20 $OUT/bench.log; exit 13; }
python -c "import json,sys; d=json.loads(open('$OUT/bench.log').read().strip().splitlines()[-1]); print(d['value'], d['roofline']['frac'], json.dumps(d['config'].get('variants')))"
