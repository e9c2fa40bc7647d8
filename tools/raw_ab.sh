#!/bin/bash
# A/B of a raw-DD kernel build variant against the product library, one box,
# alternating: parity of the variant first (the stream tests through TDBG_LIB),
# then C5 rand + ramp at the metric's 100,000 tiles.  Usage: raw_ab.sh TAG VARLIB
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-x}
V=${2:-varlibs/pw.so}
OUT=$R/gpurun_out/raw_ab_$TAG
mkdir -p $OUT
cd $R
TDBG_LIB=$V timeout -k 10 300 python -u -m pytest ${TESTS:-tests/test_gpu_c5tile.py tests/test_gpu_stream_small.py tests/test_gpu_parity.py} -m gpu -x -q --timeout 120 \
  --timeout-method thread > $OUT/pytest_variant.log 2>&1 || { echo "variant parity failed"; tail -30 $OUT/pytest_variant.log; exit 11; }
tail -1 $OUT/pytest_variant.log
for rep in 1 2; do
  for lib in base var; do
    if [ $lib = var ]; then export TDBG_LIB=$V; else unset TDBG_LIB; fi
    timeout -k 10 180 python -u bench.py --config ${CONFIG:-c5} --steps 20 --warmup 3 --variants ${VARS:-rand,ramp} --no-others --no-e2e --no-forward \
      --no-cpu-baseline --shard-tiles 0 > $OUT/${lib}_$rep.json 2> $OUT/${lib}_$rep.err \
      || { echo "bench $lib failed"; tail -20 $OUT/${lib}_$rep.err; exit 12; }
    python -c "
import json; d=json.loads([l for l in open('$OUT/${lib}_$rep.json') if l.startswith('{')][-1]); v=d['config']['variants']
print('$lib $rep', {k: (v[k]['GiBps'], v[k]['roofline_frac'], v[k]['kernel_ms']) for k in v})"
  done
done
