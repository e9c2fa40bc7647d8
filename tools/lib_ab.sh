#!/bin/bash
# Two builds of the product library on one box, alternating (TDBG_LIB):
# libtiledb_amd_old.so (a previous source state, built by hand) vs the tree's.
# usage: CFGS="c3a c3b" lib_ab.sh <tag>
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r05/libab_${1:-x}
mkdir -p $OUT
cd $R
for rep in 1 2; do
  for C in ${CFGS:-c3a c3b c4}; do
    for LIB in libtiledb_amd_old.so libtiledb_amd.so; do
      TDBG_LIB=$LIB timeout -k 10 120 python -u bench.py --config $C --steps 20 --warmup 3 --no-e2e --no-forward --no-cpu-baseline > $OUT/a.json 2> $OUT/a.err || { tail -5 $OUT/a.err; exit 11; }
      python -c "import json; d=json.loads([l for l in open('$OUT/a.json') if l.startswith('{')][-1]); r=d['roofline']; print('$C', '$LIB', 'rep $rep', d['value'], r['kernel_ms'], r['frac'])"
    done
  done
done
