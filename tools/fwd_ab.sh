#!/bin/bash
# Forward C5 (tdbg_filter_tiles on C5 active values, 12,500 tiles): the
# one-workgroup-per-tile 1024-thread kernel vs the persistent 512-thread one
# (experiments library, TDBG_FWD_PERSIST), alternating, two reps; GPU forward
# tests first.  usage: fwd_ab.sh <tag>
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r05/fwd_${1:-x}
mkdir -p $OUT
cd $R
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_forward.py -m gpu > $OUT/t.log 2>&1; rc=$?; tail -3 $OUT/t.log; [ $rc -ne 0 ] && exit $rc
export TDBG_LIB=libtiledb_amd_exp.so
for rep in 1 2; do
  for S in "X=0" "TDBG_FWD_PERSIST=1"; do
    for V in ${VARS:-active rand}; do
      env $S timeout -k 10 150 python -u bench.py --tiles-per-gpu 12500 --variants $V --steps 20 --warmup 3 --no-others --no-e2e --no-cpu-baseline --shard-tiles 0 --c5s-tiles 0 > $OUT/a.json 2> $OUT/a.err || { tail -5 $OUT/a.err; exit 11; }
      python -c "import json; d=json.loads([l for l in open('$OUT/a.json') if l.startswith('{')][-1]); f=d['forward']; print('$S $V rep $rep', f['value'], f['kernel_ms'], f['roofline_frac'])"
    done
  done
done
