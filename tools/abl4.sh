#!/bin/bash
# TDBG_C5T_ABL=4 (no general-range decoder in the kernel: every wave on the one-read path; ramp's
# plane-boundary outputs wrong, timing only) vs 0, experiments library, same box
set -o pipefail
export TDBG_LIB=libtiledb_amd_exp.so
OUT=gpurun_out/abl${TAG:-4}
mkdir -p $OUT
for rep in 1 2; do for a in ${ABLS:-0 4}; do for v in ${VARS:-ramp rand}; do
  TDBG_C5T_ABL=$a TDBG_BENCH_NOVERIFY=1 timeout -k 10 180 python -u bench.py --config c5 --steps 10 --warmup 2 --variants $v --c5s-tiles 0 --no-others --no-e2e --no-forward --no-cpu-baseline --shard-tiles 0 --legs-file= > $OUT/abl${a}_${v}_$rep.json 2> $OUT/abl${a}_${v}_$rep.err || { tail -5 $OUT/abl${a}_${v}_$rep.err; exit 11; }
  python -c "import json; d=json.loads([l for l in open('$OUT/abl${a}_${v}_$rep.json') if l.startswith('{')][-1]); print('abl=$a $v rep=$rep', d['value'], d['ms_per_step'], d['roofline']['frac'])"
done; done; done
