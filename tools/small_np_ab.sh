#!/bin/bash
# C3a / C3b / C4: the persistent 256-thread small-image kernel vs one 512-thread
# workgroup per tile (the product path; TDBG_SMALL_P: the persistent one,
# experiments build), alternating on one box.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r05/smallnp_${1:-x}
mkdir -p $OUT
cd $R
for rep in 1 2; do
  for C in ${CFGS:-c3a c3b c4}; do
    for V in ${AB:-NONE TDBG_SMALL_P}; do
      ( case $V in NONE) ;; *=*) export "$V" ;; *) export $V=1 ;; esac
        TDBG_LIB=libtiledb_amd_exp.so timeout -k 10 120 python -u bench.py --config $C --steps 20 --warmup 3 --no-e2e --no-forward --no-cpu-baseline > $OUT/a.json 2> $OUT/a.err ) || { tail -5 $OUT/a.err; exit 11; }
      python -c "import json; d=json.loads([l for l in open('$OUT/a.json') if l.startswith('{')][-1]); r=d['roofline']; print('$C', '$V', 'rep $rep', d['value'], r['kernel_ms'], r['frac'], d['config'].get('stream_tiles_timed'))"
    done
  done
done
