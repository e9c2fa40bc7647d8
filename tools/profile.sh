#!/bin/bash
# Profile bench.py on the GPU box: kernel-trace/stats pass + separate PMC passes
# (FETCH_SIZE, WRITE_SIZE) -- never combined with sys/runtime traces.
# usage: bash tools/profile.sh <tag> [bench args...]
set -o pipefail
TAG=${1:-r01}; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/prof_$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 $R/bench.py --no-cpu-baseline "$@" > $OUT/trace.log 2>&1 || exit 11
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pmc_fetch -o run -- python3 $R/bench.py --no-cpu-baseline "$@" > $OUT/pmc_fetch.log 2>&1 || exit 12
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/pmc_write -o run -- python3 $R/bench.py --no-cpu-baseline "$@" > $OUT/pmc_write.log 2>&1 || exit 13
echo done
