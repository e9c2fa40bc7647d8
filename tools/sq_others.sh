#!/bin/bash
# SQ counter passes (separate rocprofv3 --pmc runs, no traces) on the C2 tile
# kernel (C2, C2i) and the small-image kernel (C3a, C3b, C4).
# Summaries -> gpurun_out/<tag>/sq_<cfg>.json.  usage: bash tools/sq_others.sh <tag>
set -o pipefail
TAG=${1:-sqo}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
cd $R
A="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA"
C="SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS"
for CFG in ${CFGS:-c2 c2i c3a c3b c4}; do
  B="--config $CFG --no-cpu-baseline --no-e2e --no-forward --no-others --steps 10 --warmup 2"
  P=0
  for SET in "$A" "$C"; do
    P=$((P+1))
    timeout -s KILL 120 rocprofv3 --pmc $SET --output-format csv -d $OUT/sq_$CFG/pass$P -o run -- python3 $R/bench.py $B > $OUT/sq_${CFG}_$P.log 2>&1 || { echo "sq $CFG pass $P failed"; tail -20 $OUT/sq_${CFG}_$P.log; exit 12; }
  done
  case $CFG in c2|c2i) K=unfilter_c2tile_kernel ;; *) K=unfilter_stream_small_kernel ;; esac
  NT=10000; [ $CFG = c4 ] && NT=12500
  TDBG_KNAME="$K" python3 $R/tools/sq_summary.py $OUT/sq_$CFG $CFG default $NT > $OUT/sq_$CFG.json || exit 13
  echo "== $CFG ($K)"; python3 -c "import json; d=json.load(open('$OUT/sq_$CFG.json')); print(json.dumps(d['derived']))"
done
