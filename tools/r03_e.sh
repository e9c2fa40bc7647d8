#!/bin/bash
# Round-3 GPU pass e: raw-kernel timing ablations on C5 rand (TDBG_RAW_ABL:
# 1 parse once per workgroup, 2 one DMA unit per plane range, 3 no stores)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r03_${1:-e}
mkdir -p $OUT
cd $R
B="--config c5 --variants rand --no-cpu-baseline --no-e2e --no-forward --steps 20 --warmup 3"
for A in 0 1 2 3 0; do
  TDBG_BENCH_NOVERIFY=$A TDBG_RAW_ABL=$A timeout -k 10 120 python3 bench.py $B > $OUT/abl_$A.log 2>&1 || { echo "abl $A failed"; tail -20 $OUT/abl_$A.log; exit 11; }
  echo "abl $A: $(grep -o '"kernel_ms": [0-9.]*' $OUT/abl_$A.log | head -1)"
done
echo done
