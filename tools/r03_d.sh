#!/bin/bash
# Round-3 GPU pass d: persistent-grid size sweeps of the two streaming
# kernels (tail quantization: 12,500 tiles over G workgroups)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r03_${1:-d}
mkdir -p $OUT
cd $R
B="--config c5 --no-cpu-baseline --no-e2e --no-forward --steps 20 --warmup 3"
for G in 1536 1389 1280 1024 768 512; do
  TDBG_RAW_GRID=$G timeout -k 10 120 python3 bench.py $B --variants rand,ramp > $OUT/raw_$G.log 2>&1 || { echo "raw $G failed"; tail -20 $OUT/raw_$G.log; exit 11; }
  echo "raw G=$G: $(grep -o '"rand": {"GiBps": [0-9.]*, "roofline_frac": [0-9.]*, "kernel_ms": [0-9.]*' $OUT/raw_$G.log) $(grep -o '"ramp": {"GiBps": [0-9.]*, "roofline_frac": [0-9.]*, "kernel_ms": [0-9.]*' $OUT/raw_$G.log)"
done
for G in 1024 1000 962 896 768; do
  TDBG_STREAM_GRID=$G timeout -k 10 120 python3 bench.py $B --variants active > $OUT/coded_$G.log 2>&1 || { echo "coded $G failed"; tail -20 $OUT/coded_$G.log; exit 12; }
  echo "coded G=$G: $(grep -o '"kernel_ms": [0-9.]*' $OUT/coded_$G.log | head -1) $(grep -o '"frac": [0-9.]*' $OUT/coded_$G.log | head -1)"
done
echo done
