#!/bin/bash
# C2 / C2i: the bitshuffle tile kernel (tdbg_c2tile.hip) in its variants vs
# the fused kernel alone, alternating on one box (experiments build).
# AB: experiment variables to set one at a time (NONE: the product path), e.g.
#   AB="NONE TDBG_C2T_MAT TDBG_NO_C2TILE" tools/c2t_ab.sh <tag>
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r05/c2tab_${1:-x}
mkdir -p $OUT
cd $R
for rep in 1 2; do
  for C in ${CFGS:-c2 c2i}; do
    for V in ${AB:-NONE TDBG_NO_C2TILE}; do
      ( case $V in NONE) ;; *=*) export "$V" ;; *) export $V=1 ;; esac
        TDBG_LIB=libtiledb_amd_exp.so timeout -k 10 120 python -u bench.py --config $C --steps 20 --warmup 3 --no-e2e --no-forward --no-cpu-baseline > $OUT/a.json 2> $OUT/a.err ) || { tail -5 $OUT/a.err; exit 11; }
      python -c "import json; d=json.loads([l for l in open('$OUT/a.json') if l.startswith('{')][-1]); r=d['roofline']; print('$C', '$V', 'rep $rep', d['value'], r['kernel_ms'], r['frac'])"
    done
  done
done
