#!/bin/bash
# timing ablations of the raw-DD streaming kernel on C5 rand (TDBG_RAW_ABL;
# outputs not meaningful): 0 full, 2 one DMA unit per job plane, 3 no stores,
# 4 no jobs (walk + prefix + parse + barriers only)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-rawabl}
mkdir -p $OUT
cd $R
for A in 0 2 3 4; do
  TDBG_RAW_ABL=$A timeout -k 10 120 python3 -c "
import sys; sys.path.insert(0, '.')
import numpy as np, torch, bench, workloads as W
from tiledb_amd import engine
ser, dt, cs, _, _ = W.config('c5')
dp = engine.DevicePipeline(ser, 23, int(dt), cs); ctx = engine.Context(0)
batch = bench.build_batch(engine, 'c5', 'rand', 12500, 128, 0, seed=5)[0]
for _ in range(3): ctx.unfilter_async(dp, batch)
torch.cuda.synchronize()
ctx.time_launches(10)
for _ in range(10): ctx.unfilter_async(dp, batch)
torch.cuda.synchronize()
print('abl $A: launch ms', round(ctx.last_kernel_ms(), 4))
" > $OUT/abl_$A.log 2>&1 || { echo "abl $A failed"; tail -5 $OUT/abl_$A.log; exit 10; }
  grep "abl" $OUT/abl_$A.log
done
