#!/bin/bash
# Per-stage SQ instruction counts of the fused kernel by ablation:
# TDBG_DEBUG_STOP=1 (load only), 2, 3 (after the 1st / 2nd intermediate
# stage), full.  One rocprofv3 --pmc pass each (timing-only runs for 1..3).
# usage: bash tools/stage_sq.sh <tag> <config> <variant>
set -o pipefail
TAG=${1:-x}; CFG=${2:-c5}; VAR=${3:-active}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/stagesq_$TAG
mkdir -p $OUT
export TMPDIR=/tmp
cd $R
C="SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_WAVE_CYCLES SQ_WAIT_ANY"
for STOP in 1 2 3 0; do
  if [ $STOP = 0 ]; then unset TDBG_DEBUG_STOP; else export TDBG_DEBUG_STOP=$STOP; fi
  timeout -s KILL 120 rocprofv3 --pmc $C --output-format csv -d $OUT/stop$STOP -o run -- python3 $R/bench.py --config $CFG --variants $VAR --no-cpu-baseline --no-e2e --steps 5 --warmup 2 > $OUT/stop$STOP.log 2>&1 || { echo "pass $STOP failed"; tail -20 $OUT/stop$STOP.log; exit 12; }
  python3 $R/tools/sq_summary.py $OUT/stop$STOP $CFG $VAR > $OUT/stop$STOP.json || exit 13
done
python3 - <<PY
import json
rows = {s: json.load(open("$OUT/stop%s.json" % s))["counters_median_per_launch"] for s in ("1", "2", "3", "0")}
keys = sorted(rows["0"])
print("counter".ljust(24), *[("stop" + s).rjust(14) for s in ("1", "2", "3", "0")])
for k in keys:
    print(k.ljust(24), *[("%14.0f" % (rows[s].get(k, 0) / 12500)) for s in ("1", "2", "3", "0")])
PY
