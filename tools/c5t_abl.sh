#!/bin/bash
# round 5: one-workgroup-per-tile C5 kernel (tdbg_c5tile.hip) timing ablations
# against the persistent raw kernel, one box, alternating; plus the ceiling
# probe's tile shapes for calibration.  usage: c5t_abl.sh <tag>  (CFG, ABLS, VARS)
set -o pipefail
# the TDBG_* switches below exist only in the experiments library (tdbg_hooks.h)
export TDBG_LIB=${TDBG_LIB:-libtiledb_amd_exp.so}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r05/abl_${1:-x}
mkdir -p $OUT
cd $R
timeout -k 10 60 tools/ceiling3 "X b1024" > $OUT/ceiling.log 2>&1 || { echo "probe failed"; exit 12; }
for rep in 1 2; do
  for a in ${ABLS:-old 0 1 2 3}; do
    for v in ${VARS:-rand ramp}; do
      if [ $a = old ]; then ENV="TDBG_C5_OLD_RAW=1"; else ENV="TDBG_C5T_ABL=$a"; fi
      env $ENV TDBG_BENCH_NOVERIFY=1 timeout -k 10 180 python -u bench.py --config ${CFG:-c5} --steps 10 --warmup 2 --variants $v \
        --c5s-tiles 0 --no-others --no-e2e --no-forward --no-cpu-baseline --shard-tiles 0 > $OUT/abl${a}_${v}_$rep.json 2> $OUT/abl${a}_${v}_$rep.err \
        || { echo "abl $a failed"; tail -20 $OUT/abl${a}_${v}_$rep.err; exit 11; }
      python -c "import json,sys; d=json.loads([l for l in open('$OUT/abl${a}_${v}_$rep.json') if l.startswith('{')][-1]); print('abl=$a $v rep=$rep', d['value'], d['ms_per_step'], d['roofline']['frac'])"
    done
  done
done
