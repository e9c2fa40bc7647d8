#!/bin/bash
# C1 launch composition: rocprofv3 kernel trace of the C1 bench (256 tiles)
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/c1trace
mkdir -p $OUT
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/t -o run -- python3 bench.py --config c1 --variants rand --no-cpu-baseline --no-e2e --no-others --no-forward --steps 20 --warmup 3 --legs-file= > $OUT/log 2>&1 || { tail -20 $OUT/log; exit 11; }
f=$(find $OUT/t -name '*kernel_stats.csv' | head -1); cut -c1-160 $f | head -12
