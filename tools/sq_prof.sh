#!/bin/bash
# SQ counter passes (separate rocprofv3 --pmc runs, never combined with
# traces) over one bench workload; summary -> gpurun_out/sq_<tag>/sq.json
# usage: bash tools/sq_prof.sh <tag> <config> <variant>
set -o pipefail
TAG=${1:-x}; CFG=${2:-c5}; VAR=${3:-active}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/sq_$TAG
mkdir -p $OUT
export TMPDIR=/tmp
cd $R
A="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT"
B="SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SMEM"
P=0
for SET in "$A" "$B"; do
  P=$((P+1))
  timeout -s KILL 120 rocprofv3 --pmc $SET --output-format csv -d $OUT/pass$P -o run -- python3 $R/bench.py --config $CFG --variants $VAR --no-cpu-baseline --no-e2e --steps 5 --warmup 2 > $OUT/pass$P.log 2>&1 || { echo "sq pass $P failed"; tail -20 $OUT/pass$P.log; exit 12; }
done
python3 $R/tools/sq_summary.py $OUT $CFG $VAR > $OUT/sq.json || exit 13
cat $OUT/sq.json
