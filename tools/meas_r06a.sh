#!/bin/bash
# round 6 study: phase clocks of the C5 tile kernel (rand, ramp, active) and
# SQ counters on ramp (VALU share, waits) -- what holds ramp at 0.67 when its
# copy ceiling (profiles/r05/ceiling3_boxB.txt, N r43 b1024) is 0.78
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-m06a}
mkdir -p $OUT
cd $R
timeout -k 10 200 python -u tools/c5t_prof.py rand ramp > $OUT/prof_raw.txt 2>&1 || { echo "prof failed"; tail -20 $OUT/prof_raw.txt; exit 11; }
timeout -k 10 200 python -u tools/c5t_prof.py active > $OUT/prof_active.txt 2>&1 || { echo "prof failed"; tail -20 $OUT/prof_active.txt; exit 11; }
cat $OUT/prof_raw.txt $OUT/prof_active.txt | grep -v amdgpu.ids
VARS="ramp" KN=unfilter_c5tile_kernel bash tools/sq_stream.sh ${1:-m06a}/sq || exit 12
