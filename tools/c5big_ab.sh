mkdir -p gpurun_out/r05
for T in 512; do
  for CP in 0 1; do
    timeout -k 10 200 python -u - <<PY
import sys, json, time, numpy as np, torch
sys.path.insert(0, '.')
import bench, workloads as W
from tiledb_amd import engine
ctx = engine.Context(0)
ser, dt, cs, _, _ = W.config('c5big')
dp = engine.DevicePipeline(ser, 23, int(dt), cs)
batch, pool, vals, idx, packed, offs, sizes = bench.build_batch(engine, 'c5big', 'active', $T, 8, 0, seed=5, ctx=ctx, dp=dp)
st = ctx.unfilter(dp, batch, chunk_parallel=bool($CP))
assert not st.any()
s = torch.cuda.current_stream()
for _ in range(3): ctx.unfilter_async(dp, batch, stream=s.cuda_stream, chunk_parallel=bool($CP))
torch.cuda.synchronize(); t0 = time.perf_counter()
for _ in range(10): ctx.unfilter_async(dp, batch, stream=s.cuda_stream, chunk_parallel=bool($CP))
torch.cuda.synchronize(); el = (time.perf_counter() - t0) / 10
b = float(sizes.sum()) + sum(vals[i].nbytes for i in idx)
bench.verify(batch, vals, idx)
print('tiles $T chunk_parallel $CP', round(el * 1e3, 3), 'ms', round(b / el / 8e12, 4), 'frac(wall)')
PY
  done
done
