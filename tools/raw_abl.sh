#!/bin/bash
# Raw-DD kernel timing ablations at the metric's 100,000 C5 tiles (rand), one box,
# alternating: 0 = product, 4 = walk + prefix + parse + barriers only (no jobs),
# 3 = no stores.  Outputs are not meaningful under an ablation (no verify).
set -o pipefail
# the TDBG_* switches below exist only in the experiments library (tdbg_hooks.h)
export TDBG_LIB=${TDBG_LIB:-libtiledb_amd_exp.so}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/raw_abl_${1:-x}
mkdir -p $OUT
cd $R
for rep in 1 2; do
  for a in 0 4 3; do
    TDBG_RAW_ABL=$a TDBG_BENCH_NOVERIFY=1 timeout -k 10 180 python -u bench.py --steps 10 --warmup 2 --variants rand \
      --no-others --no-e2e --no-forward --no-cpu-baseline --shard-tiles 0 > $OUT/abl${a}_$rep.json 2> $OUT/abl${a}_$rep.err \
      || { echo "abl $a failed"; tail -20 $OUT/abl${a}_$rep.err; exit 11; }
    python -c "import json,sys; d=json.loads([l for l in open('$OUT/abl${a}_$rep.json') if l.startswith('{')][-1]); print('abl=$a rep=$rep', d['value'], d['ms_per_step'], d['roofline']['kernel_ms'])"
  done
done
