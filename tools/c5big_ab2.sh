#!/bin/bash
# 4 MiB C5 tiles (64 chunks of 64 KiB), one box: tile mode with the tile
# kernel's multi-chunk variant (chunk_parallel=None -> TDBG_MULTI_CHUNK) vs
# the device chunk directory (True) vs the fused kernel (False).
# usage: c5big_ab2.sh <tag>   (T=tiles, VARS=..., MODES="None True False",
# ENVS="TDBG_LIB=... ..." for another library)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/c5big_${1:-x}
mkdir -p $OUT
cd $R
for V in ${VARS:-active rand ramp}; do
for CP in ${MODES:-None True False}; do
  env $ENVS timeout -k 10 300 python -u - > $OUT/${V}_$CP.txt 2>&1 <<PY || { echo "failed $V $CP"; tail -20 $OUT/${V}_$CP.txt; exit 11; }
import sys, time, numpy as np, torch
sys.path.insert(0, '.')
import bench, workloads as W
from tiledb_amd import engine
ctx = engine.Context(0)
ser, dt, cs, _, _ = W.config('c5big')
dp = engine.DevicePipeline(ser, 23, int(dt), cs)
T = ${T:-512}
batch, pool, vals, idx, packed, offs, sizes = bench.build_batch(engine, 'c5big', '$V', T, 12, 0, seed=5, ctx=ctx, dp=dp)
k0, c0 = ctx.tile_chunks(), ctx.stream_chunks()
st = ctx.unfilter(dp, batch, chunk_parallel=$CP)
assert not st.any()
bench.verify(batch, vals, idx)
k1, c1 = ctx.tile_chunks(), ctx.stream_chunks()
s = torch.cuda.current_stream()
for _ in range(3): ctx.unfilter_async(dp, batch, stream=s.cuda_stream, chunk_parallel=$CP)
torch.cuda.synchronize(); t0 = time.perf_counter()
for _ in range(10): ctx.unfilter_async(dp, batch, stream=s.cuda_stream, chunk_parallel=$CP)
torch.cuda.synchronize(); el = (time.perf_counter() - t0) / 10
b = float(sizes.sum()) + sum(vals[i].nbytes for i in idx)
bench.verify(batch, vals, idx)
print('$V tiles', T, 'chunk_parallel=$CP', round(el * 1e3, 3), 'ms', round(b / el / 8e12, 4), 'frac(wall)',
      'tile-mode chunks', k1 - k0, 'directory chunks', c1 - c0)
PY
  tail -1 $OUT/${V}_$CP.txt
done
done
