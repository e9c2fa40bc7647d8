#!/bin/bash
# Streaming-kernel profile: kernel-trace stats of C5 active with plain and
# nontemporal stores, then the SQ counter passes (tools/sq_prof.sh layout).
set -o pipefail
# the TDBG_* switches below exist only in the experiments library (tdbg_hooks.h)
export TDBG_LIB=${TDBG_LIB:-libtiledb_amd_exp.so}
TAG=${1:-x}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/sprof_$TAG
mkdir -p $OUT
export TMPDIR=/tmp
cd $R
B="--config c5 --variants active --no-cpu-baseline --no-e2e --no-forward --steps 10 --warmup 2"
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 $R/bench.py $B > $OUT/trace.log 2>&1 || { echo "trace failed"; tail -20 $OUT/trace.log; exit 11; }
grep -h "unfilter" $OUT/trace/*kernel_stats.csv | cut -c1-160
TDBG_STREAM_NT=1 timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace_nt -o run -- python3 $R/bench.py $B > $OUT/trace_nt.log 2>&1 || { echo "trace nt failed"; tail -20 $OUT/trace_nt.log; exit 12; }
grep -h "unfilter" $OUT/trace_nt/*kernel_stats.csv | cut -c1-160
A="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT"
C="SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SMEM"
P=0
for SET in "$A" "$C"; do
  P=$((P+1))
  timeout -s KILL 120 rocprofv3 --pmc $SET --output-format csv -d $OUT/pass$P -o run -- python3 $R/bench.py $B > $OUT/pass$P.log 2>&1 || { echo "sq pass $P failed"; tail -20 $OUT/pass$P.log; exit 13; }
done
TDBG_KNAME=unfilter_stream_kernel python3 $R/tools/sq_summary.py $OUT c5 active > $OUT/sq.json || exit 14
cat $OUT/sq.json
