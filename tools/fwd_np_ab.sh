#!/bin/bash
# Forward (filter) kernels of C1 / C2 / C2i / C3a / C3b / C4: one workgroup per
# tile (product) vs the persistent grid (TDBG_FWD_P), experiments build,
# alternating on one box; prints the bench line's forward leg.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r05/fwdnp_${1:-x}
mkdir -p $OUT
cd $R
for rep in 1 2; do
  for C in ${CFGS:-c2 c2i c3a c3b c4}; do
    for V in ${AB:-NONE TDBG_FWD_P}; do
      ( case $V in NONE) ;; *=*) export "$V" ;; *) export $V=1 ;; esac
        TDBG_LIB=libtiledb_amd_exp.so timeout -k 10 120 python -u bench.py --config $C --steps 20 --warmup 3 --no-e2e --no-cpu-baseline > $OUT/a.json 2> $OUT/a.err ) || { tail -5 $OUT/a.err; exit 11; }
      python -c "import json; d=json.loads([l for l in open('$OUT/a.json') if l.startswith('{')][-1]); f=d['forward']; print('$C', '$V', 'rep $rep', f['value'], f['kernel_ms'], f['roofline_frac'])"
    done
  done
done
