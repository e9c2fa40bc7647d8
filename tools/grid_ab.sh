#!/bin/bash
# Persistent vs one-tile-per-workgroup grids for the small-image streaming
# kernel (C3a, C3b, C4) and the fused kernel (C2, C2i): experiments-library
# grid hooks, alternating, two reps.  usage: grid_ab.sh <tag>
set -o pipefail
export TDBG_LIB=libtiledb_amd_exp.so
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r05/gridab_${1:-x}
mkdir -p $OUT
cd $R
for rep in 1 2; do
  for C in ${CFGS:-c3a c3b c4 c2 c2i}; do
    for S in "X=0" "TDBG_SMALL_GRID=${NG:-10000}"; do
      env $S timeout -k 10 120 python -u bench.py --config $C --steps 20 --warmup 3 --no-e2e --no-forward --no-cpu-baseline > $OUT/ab.json 2> $OUT/ab.err || { tail -5 $OUT/ab.err; exit 11; }
      python -c "import json; d=json.loads([l for l in open('$OUT/ab.json') if l.startswith('{')][-1]); r=d['roofline']; print('$C', '$S', 'rep $rep', d['value'], d['ms_per_step'], r['kernel_ms'], r['frac'])"
    done
  done
done
