#!/bin/bash
# stream tests + phase clocks (plain and nontemporal stores) + bench
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/ph3_${1:-x}
mkdir -p $OUT
cd $R
timeout -k 10 300 python -u -m pytest tests/test_gpu_stream.py -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_stream.log 2>&1 || { echo "stream tests failed"; tail -40 $OUT/pytest_stream.log; exit 11; }
tail -1 $OUT/pytest_stream.log
for M in 0 1; do
  TDBG_STREAM_STORE=$M TDBG_PROF=1 timeout -k 10 200 python -u tools/phase_prof.py active > $OUT/phase_$M.log 2>&1 || { echo "phase $M failed"; tail -20 $OUT/phase_$M.log; exit 12; }
  echo "mode $M"; grep active $OUT/phase_$M.log
done
timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-e2e --no-forward > $OUT/bench.log 2>&1 || { echo "bench failed"; tail -20 $OUT/bench.log; exit 13; }
python -c "import json,sys; d=json.loads(open('$OUT/bench.log').read().strip().splitlines()[-1]); print(d['value'], d['roofline']['frac'], json.dumps(d['config'].get('variants')))"
