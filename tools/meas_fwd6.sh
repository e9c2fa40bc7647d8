#!/bin/bash
# round 6: forward C5 tile kernel phase clocks (active, rand) and SQ counters (active)
set -o pipefail
OUT=gpurun_out/fwd6
mkdir -p $OUT
timeout -k 10 300 python -u tools/phase_prof_fwd.py active rand > $OUT/phase.txt 2>&1 || { tail -20 $OUT/phase.txt; exit 11; }
grep -v amdgpu.ids $OUT/phase.txt
bash tools/sq_fwd.sh fwd6/sq || exit 12
