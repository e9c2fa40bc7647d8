#!/bin/bash
# Same-box A/B of whole libraries (tools/build_variant.sh), alternating, 2
# reps: LIBS="libtiledb_amd_base.so libtiledb_amd.so" VARS="rand ramp active"
# CFG=c5 [TILES=n] [ENVS="X=1"] bash tools/ab_lib.sh <tag>
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/abl_${1:-x}
mkdir -p $OUT
cd $R
TP=""; [ -n "$TILES" ] && TP="--tiles-per-gpu $TILES"
for rep in 1 2; do
  for L in ${LIBS:-libtiledb_amd_base.so libtiledb_amd.so}; do
    for v in ${VARS:-rand ramp active}; do
      E="TDBG_LIB=$L"; [ "$L" = libtiledb_amd.so ] && E="TDBG_NONE=1"
      env $E $ENVS timeout -k 10 180 python -u bench.py --config ${CFG:-c5} --steps 10 --warmup 2 --variants $v $TP \
        --c5s-tiles 0 --no-others --no-e2e --no-forward --no-cpu-baseline --shard-tiles 0 --legs-file '' > $OUT/${L}_${v}_$rep.json 2> $OUT/${L}_${v}_$rep.err \
        || { echo "$L $v failed"; tail -20 $OUT/${L}_${v}_$rep.err; exit 11; }
      python -c "import json; d=json.loads(open('$OUT/${L}_${v}_$rep.json').read().strip().splitlines()[-1]); print('$L $v rep=$rep', d['value'], d['ms_per_step'], d['roofline']['frac'])"
    done
  done
done
