#!/bin/bash
# Round-3 GPU pass j: E2E regression hunt -- the same bench command at 20 and
# 5 timed steps (forward leg on), and e2e-only runs with the process bound to
# the GPU's NUMA node vs not (first-touch placement of the pinned buffers)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r03_${1:-j}
mkdir -p $OUT
cd $R
for S in 20 5 20; do
  timeout -k 10 300 python3 bench.py --no-cpu-baseline --steps $S --warmup 3 > $OUT/e2e_s$S.log 2>&1 || { echo "bench s$S failed"; tail -20 $OUT/e2e_s$S.log; exit 11; }
  echo "steps $S: $(grep -o '"e2e_GiBps": {[^}]*}' $OUT/e2e_s$S.log)"
done
timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-forward --steps 20 --warmup 3 > $OUT/e2e_nofwd20.log 2>&1 || { echo "bench nofwd failed"; exit 12; }
echo "steps 20 no forward: $(grep -o '"e2e_GiBps": {[^}]*}' $OUT/e2e_nofwd20.log)"
echo done
