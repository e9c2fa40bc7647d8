#!/bin/bash
# Kernel timeline of a chunk-parallel C5 launch (512 tiles of 4 MiB, 64 chunks each)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r05/c5big_${1:-x}
mkdir -p $OUT
export TMPDIR=/tmp
cd $R
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 $R/bench.py --config c5big --tiles-per-gpu ${TILES:-512} --variants active --steps 10 --warmup 2 --no-e2e --no-forward --no-cpu-baseline > $OUT/b.log 2>&1 || { tail -5 $OUT/b.log; exit 11; }
tail -1 $OUT/b.log | cut -c1-300
python3 $R/tools/gap_summary.py $OUT/trace 14
