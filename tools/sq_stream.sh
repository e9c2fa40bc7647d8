#!/bin/bash
# SQ counter passes (separate rocprofv3 --pmc runs, no traces) on the two
# streaming kernels: unfilter_stream_raw_kernel over C5 rand and
# unfilter_stream_kernel over C5 active.  Summaries -> gpurun_out/<tag>/sq_*.json
# usage: bash tools/sq_stream.sh <tag>   (VARS=..., KN=<kernel name substring>)
set -o pipefail
TAG=${1:-sq}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
cd $R
A="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA"
C="SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS"
for V in ${VARS:-rand active}; do
  B="--config c5 --variants $V --no-cpu-baseline --no-e2e --no-forward --no-others --shard-tiles 0 --steps 10 --warmup 2"
  P=0
  for SET in "$A" "$C"; do
    P=$((P+1))
    timeout -s KILL 120 rocprofv3 --pmc $SET --output-format csv -d $OUT/sq_$V/pass$P -o run -- python3 $R/bench.py $B > $OUT/sq_${V}_$P.log 2>&1 || { echo "sq $V pass $P failed"; tail -20 $OUT/sq_${V}_$P.log; exit 12; }
  done
  K=${KN:-$([ $V = rand ] && echo unfilter_stream_raw_kernel || echo "unfilter_stream_kernel<")}
  TDBG_KNAME="$K" python3 $R/tools/sq_summary.py $OUT/sq_$V c5 $V ${SQ_TILES:-100000} > $OUT/sq_$V.json || exit 13
  echo "== $V ($K)"; python3 -c "import json; d=json.load(open('$OUT/sq_$V.json')); print(json.dumps(d['derived'])); c=d['counters_median_per_launch']; print({k: c[k] for k in sorted(c)})"
done
