"""Per-phase cycle breakdown of the LDS-resident C5 forward kernel
(tdbg_forward_stream.hip, TDBG_PROF=1).  Run on the GPU box:
    TDBG_PROF=1 python tools/phase_prof_fwd.py [active rand ramp]"""
import os
import sys

os.environ.setdefault("TDBG_PROF", "1")
os.environ.setdefault("TDBG_LIB", "libtiledb_amd_exp.so")  # (hooks: experiments library)
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np
import torch

import bench
import workloads as W
from tiledb_amd import engine

NAMES = ["loads+transposes", "bitsize+B1", "dd-output+B2", "bwr-windows+B3", "scan+headers+B4/B5",
         "compress+B6", "store"]
_ser, _dt, _cs, _, _ = W.config("c5")
dp = engine.DevicePipeline(_ser, 23, int(_dt), _cs)
ctx = engine.Context(0)
for var in sys.argv[1:] or ["active"]:
    batch, pool, vals, idx, *_ = bench.build_batch(engine, "c5", var, 12500, 128, 0, seed=5, ctx=ctx, dp=dp)
    del batch
    fb = ctx.filter_batch(dp, [vals[i] for i in idx])
    s = torch.cuda.current_stream()
    for _ in range(3):
        ctx.filter_async(dp, fb, stream=s.cuda_stream)
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record(s)
    ctx.filter_async(dp, fb, stream=s.cuda_stream)
    b.record(s)
    torch.cuda.synchronize()
    clk = ctx.phase_clocks(8).astype(np.float64)[: len(NAMES)]
    tot = clk.sum()
    print(f"{var}: launch {a.elapsed_time(b):.4f} ms; per-WG phase share:",
          ", ".join(f"{n} {100 * c / tot:.1f}%" for n, c in zip(NAMES, clk)), flush=True)
    del fb
    torch.cuda.empty_cache()
