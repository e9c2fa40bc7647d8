#!/bin/bash
# Round-3 GPU pass b: stream-kernel tests after the barrier hardening, plain
# vs nontemporal stores on C5 active, kernel traces of C5 rand/ramp, and the
# E2E rate with and without the forward leg in the same process (regression
# hunt), with the GPU's NUMA node.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r03_${1:-b}
mkdir -p $OUT
export TMPDIR=/tmp
cd $R
for d in /sys/bus/pci/devices/*; do
  c=$(cat $d/class 2>/dev/null)
  if [ "$c" = "0x120000" ] || [ "$c" = "0x038000" ]; then echo "$d numa=$(cat $d/numa_node) cpus=$(cat $d/local_cpulist)"; fi
done > $OUT/numa.log
cat $OUT/numa.log; python3 -c "import os; print('affinity', len(os.sched_getaffinity(0)), sorted(os.sched_getaffinity(0))[:4], '...')"
timeout -k 10 300 python -u -m pytest tests/test_gpu_stream.py -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_stream.log 2>&1 || { echo "pytest failed"; tail -40 $OUT/pytest_stream.log; exit 11; }
tail -2 $OUT/pytest_stream.log
B="--config c5 --variants active --no-cpu-baseline --no-e2e --no-forward --steps 20 --warmup 3"
for rep in 1 2; do
  for M in 0 1; do
    TDBG_STREAM_STORE=$M timeout -k 10 120 python3 bench.py $B > $OUT/st_${M}_$rep.log 2>&1 || { echo "store $M failed"; tail -20 $OUT/st_${M}_$rep.log; exit 12; }
    echo "store mode $M rep $rep: $(grep -o '"roofline_frac": [0-9.]*' $OUT/st_${M}_$rep.log | head -1) $(grep -o '"ms_per_step": [0-9.]*' $OUT/st_${M}_$rep.log | head -1)"
  done
done
for V in rand ramp; do
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace_$V -o run -- python3 $R/bench.py --config c5 --variants $V --no-cpu-baseline --no-e2e --no-forward --steps 10 --warmup 2 > $OUT/trace_$V.log 2>&1 || { echo "trace $V failed"; tail -20 $OUT/trace_$V.log; exit 13; }
  echo "== $V"; grep -h "unfilter\|fixup" $OUT/trace_$V/*kernel_stats.csv | cut -c1-150
done
timeout -k 10 300 python3 bench.py --no-cpu-baseline --steps 5 --warmup 2 > $OUT/e2e_fwd.log 2>&1 || { echo "e2e fwd failed"; tail -20 $OUT/e2e_fwd.log; exit 14; }
echo "with forward:"; grep -o '"e2e_GiBps": {[^}]*}' $OUT/e2e_fwd.log
timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-forward --steps 5 --warmup 2 > $OUT/e2e_nofwd.log 2>&1 || { echo "e2e nofwd failed"; tail -20 $OUT/e2e_nofwd.log; exit 15; }
echo "no forward:"; grep -o '"e2e_GiBps": {[^}]*}' $OUT/e2e_nofwd.log
echo done
