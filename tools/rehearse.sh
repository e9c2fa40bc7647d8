#!/bin/bash
# 2-rank rehearsal of bench.py's multi-rank path (gloo; both ranks on the box's one GPU)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/rehearse_${1:-x}
mkdir -p $OUT
cd $R
TDBG_DIST_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29513 bench.py --gpus 2 --steps 5 --warmup 2 --no-cpu-baseline --no-e2e --no-forward > $OUT/bench_2rank.log 2>&1 || { echo "2-rank rehearsal failed"; tail -30 $OUT/bench_2rank.log; exit 13; }
grep '^{' $OUT/bench_2rank.log | tail -1 | cut -c1-600
