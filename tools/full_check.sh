#!/bin/bash
# Full GPU pass: every -m gpu test, smoke, the default bench line, and a
# 2-rank rehearsal of bench.py's multi-rank path (gloo, both ranks on the one
# GPU of the box).  Each GPU step time-limited, chained.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/full_${1:-x}
mkdir -p $OUT
cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -40 $OUT/pytest_gpu.log; exit 11; }
tail -2 $OUT/pytest_gpu.log
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { echo "smoke failed"; tail -30 $OUT/smoke.log; exit 12; }
tail -2 $OUT/smoke.log
TDBG_DIST_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29513 bench.py --gpus 2 --steps 5 --warmup 2 --no-cpu-baseline --no-e2e --no-forward > $OUT/bench_2rank.log 2>&1 || { echo "2-rank rehearsal failed"; tail -30 $OUT/bench_2rank.log; exit 13; }
grep '^{' $OUT/bench_2rank.log | tail -1 | cut -c1-400
