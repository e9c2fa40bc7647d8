#!/bin/bash
# C1 shuffle kernel A/B (header and plane loads issued together vs the header
# first): the GPU suite on the product library, then bench --config c1 on the
# current library and on a saved copy of the previous one, alternating, one box.
# usage: c1_ab.sh <tag> <old library basename>
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r05/c1ab_${1:-x}
mkdir -p $OUT
cd $R
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -30 $OUT/pytest_gpu.log; exit 10; }
tail -1 $OUT/pytest_gpu.log
for rep in 1 2 3; do
  for lib in new old; do
    if [ $lib = old ]; then export TDBG_LIB=$2; else unset TDBG_LIB; fi
    timeout -k 10 180 python -u bench.py --config c1 --steps 50 --warmup 5 --no-e2e --no-forward --no-cpu-baseline \
      > $OUT/${lib}_$rep.json 2> $OUT/${lib}_$rep.err || { echo "$lib failed"; tail -20 $OUT/${lib}_$rep.err; exit 11; }
    python -c "import json; d=json.loads([l for l in open('$OUT/${lib}_$rep.json') if l.startswith('{')][-1]); r=d['roofline']; print('$lib rep=$rep', d['value'], d['ms_per_step'], r['kernel_ms'], r['frac'])"
  done
done
