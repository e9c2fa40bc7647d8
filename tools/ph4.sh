#!/bin/bash
# phase clocks: default vs no-store ablation (TDBG_STREAM_STORE=3, timing only)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/ph4_${1:-x}
mkdir -p $OUT
cd $R
for M in 0 3; do
  TDBG_STREAM_STORE=$M TDBG_PROF=1 timeout -k 10 200 python -u tools/phase_prof.py active > $OUT/phase_$M.log 2>&1 || { echo "phase $M failed"; tail -20 $OUT/phase_$M.log; exit 12; }
  echo "mode $M"; grep active $OUT/phase_$M.log
done
