#!/bin/bash
# Quick GPU-box iteration: GPU parity suite, then phase clocks and a short
# bench of the C5 variants.  Each GPU step time-limited, chained with &&.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/quick_${1:-x}
mkdir -p $OUT
cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -40 $OUT/pytest_gpu.log; exit 11; }
tail -2 $OUT/pytest_gpu.log
TDBG_PROF=1 timeout -k 10 200 python -u tools/phase_prof.py active rand ramp > $OUT/phase.log 2>&1 || { echo "phase failed"; tail -20 $OUT/phase.log; exit 12; }
grep launch $OUT/phase.log
timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-e2e ${BENCH_ARGS} > $OUT/bench.log 2>&1 || { echo "bench failed"; tail -20 $OUT/bench.log; exit 13; }
python -c "import json,sys; d=json.loads(open('$OUT/bench.log').read().strip().splitlines()[-1]); print(d['value'], d['roofline']['frac'], json.dumps(d['config'].get('variants')))"
