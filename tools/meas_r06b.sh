#!/bin/bash
# round 6: phase clocks + SQ counters of the C5 tile kernel on 'active' after
# the all-zero-codes wave path (what now holds active)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-m06b}
mkdir -p $OUT
cd $R
timeout -k 10 200 python -u tools/c5t_prof.py active > $OUT/prof_active.txt 2>&1 || { echo "prof failed"; tail -20 $OUT/prof_active.txt; exit 11; }
grep -v amdgpu.ids $OUT/prof_active.txt
VARS="active" KN=unfilter_c5tile_kernel bash tools/sq_stream.sh ${1:-m06b}/sq || exit 12
