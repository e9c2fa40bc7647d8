#!/bin/bash
# rocprofv3 kernel trace of the 12,500-tile C5 shard (one GPU's share of the
# 8-GPU config): the dispatch timeline of a step (tile kernel, fused kernel on
# its queue, fixup) and the gaps between them -> gpurun_out/r05/gap_<tag>/
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r05/gap_${1:-x}
mkdir -p $OUT
export TMPDIR=/tmp
cd $R
for V in ${VARS:-rand}; do
  timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $OUT/trace_$V -o run -- python3 $R/bench.py --config c5 --tiles-per-gpu ${TILES:-12500} --variants $V --no-cpu-baseline --no-e2e --no-forward --no-others --steps 20 --warmup 3 > $OUT/trace_$V.log 2>&1 || { echo "trace $V failed"; tail -20 $OUT/trace_$V.log; exit 12; }
  tail -1 $OUT/trace_$V.log | cut -c1-300
done
