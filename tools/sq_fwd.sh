#!/bin/bash
# SQ counter passes (separate rocprofv3 --pmc runs) on the C5 forward kernel
set -o pipefail
TAG=${1:-sqf}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
cd $R
A="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA"
C="SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS"
B="--config c5 --variants active --tiles-per-gpu 12500 --no-cpu-baseline --no-e2e --no-others --steps 5 --warmup 2"
P=0
for SET in "$A" "$C"; do
  P=$((P+1))
  timeout -s KILL 120 rocprofv3 --pmc $SET --output-format csv -d $OUT/sq_fwd/pass$P -o run -- python3 $R/bench.py $B > $OUT/sq_fwd_$P.log 2>&1 || { echo "sq pass $P failed"; tail -20 $OUT/sq_fwd_$P.log; exit 12; }
done
TDBG_KNAME="${KN:-fws::filter_c5tile_kernel}" python3 $R/tools/sq_summary.py $OUT/sq_fwd c5 active > $OUT/sq_fwd.json || exit 13
python3 -c "import json; d=json.load(open('$OUT/sq_fwd.json')); print(json.dumps(d['derived']))"
