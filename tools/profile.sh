#!/bin/bash
# Profile bench.py on the GPU box (MI355X_MICROARCH.md "HBM" recipe):
#   1. rocprofv3 --kernel-trace --stats over the default bench command
#   2. separate --pmc passes (FETCH_SIZE, then WRITE_SIZE) per data variant --
#      never combined with sys/runtime/memory traces
#   3. tools/pmc_summary.py -> gpurun_out/prof_<tag>/pmc_traffic.json
# usage: bash tools/profile.sh <tag>
set -o pipefail
TAG=${1:-r01}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/prof_$TAG
mkdir -p $OUT
export TMPDIR=/tmp
cd $R
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 $R/bench.py --no-cpu-baseline --no-e2e > $OUT/trace.log 2>&1 || { echo "trace pass failed"; tail -20 $OUT/trace.log; exit 11; }
for V in rand ramp; do
  for C in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 120 rocprofv3 --pmc $C --output-format csv -d $OUT/pmc_${V}_$C -o run -- python3 $R/bench.py --no-cpu-baseline --no-e2e --variants $V --steps 10 --warmup 2 > $OUT/pmc_${V}_$C.log 2>&1 || { echo "pmc pass $V $C failed"; tail -20 $OUT/pmc_${V}_$C.log; exit 12; }
  done
done
python3 $R/tools/pmc_summary.py $OUT > $OUT/pmc_traffic.json || exit 13
cat $OUT/pmc_traffic.json
grep -h "unfilter" $OUT/trace/*kernel_stats.csv
echo done
