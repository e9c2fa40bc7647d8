#!/bin/bash
# One GPU-box pass for a round: every -m gpu test, smoke, the default bench
# line (the driver's command; compact last line + legs side file), and a
# 2-rank rehearsal of bench.py's multi-rank path (gloo, both ranks on the one
# GPU).  Each GPU step time-limited, chained; stops at the first failure.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/rc_${1:-x}
mkdir -p $OUT
cd $R
if [ -z "$SKIP_TESTS" ]; then
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -40 $OUT/pytest_gpu.log; exit 11; }
tail -2 $OUT/pytest_gpu.log
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { echo "smoke failed"; tail -30 $OUT/smoke.log; exit 12; }
tail -2 $OUT/smoke.log
fi
timeout -k 10 400 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 --legs-file $OUT/bench_legs.json > $OUT/bench.log 2>&1 || { echo "bench failed"; tail -30 $OUT/bench.log; exit 13; }
tail -1 $OUT/bench.log | wc -c
tail -1 $OUT/bench.log | cut -c1-1500
if [ -z "$SKIP_2RANK" ]; then
TDBG_DIST_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29513 bench.py --gpus 2 --steps 5 --warmup 2 --no-cpu-baseline --no-e2e --no-forward --legs-file '' > $OUT/bench_2rank.log 2>&1 || { echo "2-rank rehearsal failed"; tail -30 $OUT/bench_2rank.log; exit 13; }
tail -1 $OUT/bench_2rank.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('2rank', d['n_gpus'], d['value'], r['frac'], r['traffic']/r['algorithmic_bytes_per_launch'], r['traffic_source'])"
fi
