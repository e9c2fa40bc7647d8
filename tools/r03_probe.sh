#!/bin/bash
# Round-3 first GPU pass: HBM ceilings for the unfilter access shape, PCIe
# probe, the default bench line, E2E at several staging batch sizes, and SQ
# counter passes on unfilter_stream_kernel (C5 active).  Every GPU step has
# its own time limit; steps are chained (&&-style via exit codes).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r03_${1:-a}
mkdir -p $OUT
export TMPDIR=/tmp
cd $R
timeout -k 10 120 ./tools/ceiling > $OUT/ceiling.log 2>&1 || { echo "ceiling failed"; tail $OUT/ceiling.log; exit 10; }
cat $OUT/ceiling.log
timeout -k 10 120 python3 tools/pcie_probe.py > $OUT/pcie.log 2>&1 || { echo "pcie failed"; tail $OUT/pcie.log; exit 11; }
cat $OUT/pcie.log
timeout -k 10 300 python3 bench.py > $OUT/bench.log 2>&1 || { echo "bench failed"; tail -30 $OUT/bench.log; exit 12; }
grep '^{' $OUT/bench.log | cut -c1-1500
for MB in 16 64 256; do
  timeout -k 10 200 python3 bench.py --config c5 --variants rand,ramp --no-forward --no-cpu-baseline --steps 3 --warmup 1 --e2e-batch-mb $MB > $OUT/e2e_$MB.log 2>&1 || { echo "e2e $MB failed"; tail -30 $OUT/e2e_$MB.log; exit 13; }
  echo "batch $MB MiB:"; grep -o '"e2e_GiBps": {[^}]*}' $OUT/e2e_$MB.log
done
TDBG_NO_STREAM=1 timeout -k 10 200 python3 bench.py --config c5 --variants rand,ramp --no-forward --no-cpu-baseline --steps 3 --warmup 1 > $OUT/e2e_nostream.log 2>&1 || { echo "e2e nostream failed"; exit 14; }
echo "no stream:"; grep -o '"e2e_GiBps": {[^}]*}' $OUT/e2e_nostream.log
TDBG_DEBUG_TILE_MODE=1 timeout -k 10 200 python3 bench.py --config c5 --variants rand,ramp --no-forward --no-cpu-baseline --steps 3 --warmup 1 > $OUT/e2e_tilemode.log 2>&1 || { echo "e2e tilemode failed"; exit 15; }
echo "tile mode:"; grep -o '"e2e_GiBps": {[^}]*}' $OUT/e2e_tilemode.log
B="--config c5 --variants active --no-cpu-baseline --no-e2e --no-forward --steps 10 --warmup 2"
A="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT"
C="SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVES"
P=0
for SET in "$A" "$C"; do
  P=$((P+1))
  timeout -s KILL 120 rocprofv3 --pmc $SET --output-format csv -d $OUT/sq/pass$P -o run -- python3 $R/bench.py $B > $OUT/sq_pass$P.log 2>&1 || { echo "sq pass $P failed"; tail -20 $OUT/sq_pass$P.log; exit 16; }
done
TDBG_KNAME=unfilter_stream_kernel python3 $R/tools/sq_summary.py $OUT/sq c5 active > $OUT/sq_stream.json || exit 17
cat $OUT/sq_stream.json
echo done
