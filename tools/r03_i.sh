#!/bin/bash
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r03_${1:-i}
mkdir -p $OUT
cd $R
B="--config c5 --variants rand --no-cpu-baseline --no-e2e --no-forward --steps 20 --warmup 3"
for A in 0 1 4 2 3; do
  TDBG_BENCH_NOVERIFY=1 TDBG_RAW_ABL=$A timeout -k 10 120 python3 bench.py $B > $OUT/abl_$A.log 2>&1 || { echo "abl $A failed"; tail -20 $OUT/abl_$A.log; exit 13; }
  echo "abl $A: $(grep -o '"kernel_ms": [0-9.]*' $OUT/abl_$A.log | head -1)"
done
