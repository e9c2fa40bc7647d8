#!/bin/bash
# Round-5 final measurements: every GPU test, smoke, the default bench line,
# rocprofv3 kernel traces + PMC traffic for C5 (100k), its 12,500-tile shard
# and 40,000-B tiles.  Outputs under gpurun_out/r05/final_<tag>/
set -o pipefail
T=${1:-a}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r05/final_$T
mkdir -p $OUT
cd $R
timeout -k 10 600 python -u -m pytest -x -q --timeout 180 --timeout-method thread tests -m gpu > $OUT/t_gpu.log 2>&1; rc=$?; tail -2 $OUT/t_gpu.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail -5 $OUT/smoke.log; exit 2; }
tail -1 $OUT/smoke.log
timeout -k 10 900 python -u bench.py --steps 20 --warmup 5 > $OUT/bench_default.json 2> $OUT/bench_default.err || { tail -5 $OUT/bench_default.err; exit 3; }
BARGS="--no-cpu-baseline --no-e2e --no-forward --no-others --shard-tiles 0 --c5s-tiles 0" bash tools/profile_all.sh r05final_$T c5 c5shard c5s > $OUT/prof.log 2>&1 || { tail -5 $OUT/prof.log; exit 4; }
echo done
