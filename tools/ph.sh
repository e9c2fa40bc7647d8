#!/bin/bash
# stream tests, phase clocks and a C5 bench of the streaming kernel
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/ph_${1:-x}
mkdir -p $OUT
cd $R
timeout -k 10 300 python -u -m pytest tests/test_gpu_stream.py -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_stream.log 2>&1 || { echo "stream tests failed"; tail -40 $OUT/pytest_stream.log; exit 11; }
tail -1 $OUT/pytest_stream.log
TDBG_PROF=1 timeout -k 10 200 python -u tools/phase_prof.py active > $OUT/phase.log 2>&1 || { echo "phase failed"; tail -20 $OUT/phase.log; exit 12; }
tail -2 $OUT/phase.log
timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-e2e --no-forward > $OUT/bench.log 2>&1 || { echo "bench failed"; tail -20 $OUT/bench.log; exit 13; }
python -c "import json,sys; d=json.loads(open('$OUT/bench.log').read().strip().splitlines()[-1]); print(d['value'], d['roofline']['frac'], json.dumps(d['config'].get('variants')))"
export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 $R/bench.py --no-cpu-baseline --no-e2e --no-forward --steps 10 --warmup 2 > $OUT/trace.log 2>&1 || { echo "trace failed"; tail -20 $OUT/trace.log; exit 14; }
grep -h "unfilter" $OUT/trace/*kernel_stats.csv | cut -c1-120
