#!/bin/bash
# Per-step dispatch overhead on the 12,500-tile C5 shard under grid settings
# of the fused-on-queue and fixup dispatches (experiments library hooks):
# ms_per_step vs the events' kernel time, alternating, two reps.
set -o pipefail
export TDBG_LIB=libtiledb_amd_exp.so
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r05/gapab_${1:-x}
mkdir -p $OUT
cd $R
for rep in 1 2; do
  for S in "X=0" "TDBG_FIXUP_GRID=1" "TDBG_QGRID=64" "TDBG_QGRID=64 TDBG_FIXUP_GRID=1"; do
    env $S timeout -k 10 120 python -u bench.py --config c5 --tiles-per-gpu 12500 --variants ${V:-rand} --steps 40 --warmup 5 \
      --no-others --no-e2e --no-forward --no-cpu-baseline > $OUT/ab.json 2> $OUT/ab.err || { tail -5 $OUT/ab.err; exit 11; }
    python -c "import json; d=json.loads([l for l in open('$OUT/ab.json') if l.startswith('{')][-1]); r=d['roofline']; print('$S rep $rep', d['ms_per_step'], r['kernel_ms'], r['launch_ms'], round((d['ms_per_step']-r['kernel_ms'])*1e3,1), 'us')"
  done
done
