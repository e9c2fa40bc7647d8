#!/bin/bash
# phase clocks of the streaming kernel for each store mode (TDBG_STREAM_STORE)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/ph2_${1:-x}
mkdir -p $OUT
cd $R
for M in 0 1; do
  TDBG_STREAM_STORE=$M TDBG_PROF=1 timeout -k 10 200 python -u tools/phase_prof.py active > $OUT/phase_$M.log 2>&1 || { echo "phase $M failed"; tail -20 $OUT/phase_$M.log; exit 12; }
  echo "mode $M"; grep active $OUT/phase_$M.log
done
