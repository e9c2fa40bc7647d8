#!/bin/bash
# Same-box A/B of the C5 tile kernel's experiment variants (TDBG_C5T_ABL,
# experiments library), alternating, 2 reps each.  usage: ab_c5t.sh <tag>
# (ABLS="0 7", VARS="ramp rand", CFG=c5, TILES=<tiles per launch, default the config's>)
set -o pipefail
export TDBG_LIB=${TDBG_LIB:-libtiledb_amd_exp.so}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/ab_${1:-x}
mkdir -p $OUT
cd $R
TP=""; [ -n "$TILES" ] && TP="--tiles-per-gpu $TILES"
for rep in 1 2; do
  for a in ${ABLS:-0 7}; do
    for v in ${VARS:-ramp rand}; do
      NV=""; [ "$a" = 1 -o "$a" = 2 -o "$a" = 3 -o "$a" = 4 -o "$a" = 5 -o "$a" = 6 ] && NV="TDBG_BENCH_NOVERIFY=1"
      env TDBG_C5T_ABL=$a $NV timeout -k 10 180 python -u bench.py --config ${CFG:-c5} --steps 10 --warmup 2 --variants $v $TP \
        --c5s-tiles 0 --no-others --no-e2e --no-forward --no-cpu-baseline --shard-tiles 0 --legs-file '' > $OUT/abl${a}_${v}_$rep.json 2> $OUT/abl${a}_${v}_$rep.err \
        || { echo "abl $a failed"; tail -20 $OUT/abl${a}_${v}_$rep.err; exit 11; }
      python -c "import json,sys; d=json.loads(open('$OUT/abl${a}_${v}_$rep.json').read().strip().splitlines()[-1]); print('abl=$a $v rep=$rep', d['value'], d['ms_per_step'], d['roofline']['frac'])"
    done
  done
done
