#!/bin/bash
# Every BASELINE config on the GPU box: one bench JSON line per config
# (default variants, CPU baseline on a bounded sample), then per (config,
# variant) a rocprofv3 --kernel-trace --stats pass and separate --pmc
# FETCH_SIZE / WRITE_SIZE passes (MI355X_MICROARCH.md "HBM"); summary ->
# gpurun_out/prof_<tag>/summary.json
# usage: bash tools/profile_all.sh <tag> [configs...]   (BARGS: the bench line's extra arguments)
set -o pipefail
TAG=${1:-x}; shift
CFGS=${@:-"c5 c1 c2 c2i c3a c3b c4"}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/prof_$TAG
mkdir -p $OUT
export TMPDIR=/tmp
cd $R
declare -A VARS=([c1]="ramp rand" [c2]="sin" [c2i]="sin" [c3a]="coords" [c3b]="coords" [c4]="offsets" [c5]="active rand ramp" [xor]="sin" [delta]="active" [fscale]="sin" [c5big]="active rand ramp" [c5s]="active rand ramp" [c5shard]="active rand ramp")
for CFG in $CFGS; do
  # c5shard: C5 on one GPU's shard of the 8-GPU config (12,500 tiles)
  if [ $CFG = c5shard ]; then CA="--config c5 --tiles-per-gpu 12500"; else CA="--config $CFG"; fi
  timeout -k 10 200 python3 -u bench.py $CA ${BARGS:---cpu-seconds 5} > $OUT/bench_$CFG.log 2>&1 || { echo "bench $CFG failed"; tail -20 $OUT/bench_$CFG.log; exit 11; }
  tail -1 $OUT/bench_$CFG.log
  for V in ${VARS[$CFG]}; do
    B="$R/bench.py $CA --variants $V --no-cpu-baseline --no-e2e --no-others --no-forward"
    timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace_${CFG}_$V -o run -- python3 $B --steps 20 --warmup 3 > $OUT/trace_${CFG}_$V.log 2>&1 || { echo "trace $CFG $V failed"; tail -20 $OUT/trace_${CFG}_$V.log; exit 12; }
    for C in FETCH_SIZE WRITE_SIZE; do
      timeout -s KILL 120 rocprofv3 --pmc $C --output-format csv -d $OUT/pmc_${CFG}_${V}_$C -o run -- python3 $B --steps 10 --warmup 2 > $OUT/pmc_${CFG}_${V}_$C.log 2>&1 || { echo "pmc $CFG $V $C failed"; tail -20 $OUT/pmc_${CFG}_${V}_$C.log; exit 13; }
    done
  done
done
python3 $R/tools/profile_summary.py $OUT > $OUT/summary.json || exit 14
echo summary written
