#!/bin/bash
# Does the relative placement of the filtered tiles and the outputs in the
# bench's arena move the C5 rate?  (layout experiments, one process each)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r05/arena_${1:-x}
mkdir -p $OUT
cd $R
for S in ${SETS:-"X=0"}; do
  env $S timeout -k 10 200 python -u bench.py --variants ${V:-rand,ramp} --steps 10 --warmup 2 --no-others --no-e2e --no-forward --no-cpu-baseline --shard-tiles 0 --c5s-tiles 0 > $OUT/a.json 2> $OUT/a.err || { tail -5 $OUT/a.err; exit 11; }
  python -c "import json; d=json.loads([l for l in open('$OUT/a.json') if l.startswith('{')][-1]); v=d['config']['variants']; print('$S', {k: v[k]['roofline_frac'] for k in v})"
done
