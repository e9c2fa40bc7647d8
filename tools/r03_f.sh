#!/bin/bash
# Round-3 GPU pass f: streaming tests, then C5 rand/ramp timing + raw ablations
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r03_${1:-f}
mkdir -p $OUT
cd $R
timeout -k 10 400 python -u -m pytest tests/test_gpu_stream.py -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_stream.log 2>&1 || { echo "pytest failed"; tail -40 $OUT/pytest_stream.log; exit 11; }
tail -2 $OUT/pytest_stream.log
B="--config c5 --no-cpu-baseline --no-e2e --no-forward --steps 20 --warmup 3"
timeout -k 10 120 python3 bench.py $B --variants rand,ramp,active > $OUT/bench.log 2>&1 || { echo "bench failed"; tail -20 $OUT/bench.log; exit 12; }
grep -o '"variants": {.*}}, "min' $OUT/bench.log
for A in 2 3; do
  TDBG_BENCH_NOVERIFY=1 TDBG_RAW_ABL=$A timeout -k 10 120 python3 bench.py $B --variants rand > $OUT/abl_$A.log 2>&1 || { echo "abl $A failed"; tail -20 $OUT/abl_$A.log; exit 13; }
  echo "abl $A: $(grep -o '"kernel_ms": [0-9.]*' $OUT/abl_$A.log | head -1)"
done
echo done
