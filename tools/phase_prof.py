"""Per-phase cycle breakdown of the fused kernel on the C5 bench workload.
Run on the GPU box:  TDBG_PROF=1 python tools/phase_prof.py"""
import os, sys
os.environ.setdefault("TDBG_PROF", "1")
os.environ.setdefault("TDBG_LIB", "libtiledb_amd_exp.so")  # (hooks: experiments library)
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np
import torch
import bench
import workloads as W
from tiledb_amd import engine

NAMES = ["wait", "headers", "stage-a", "stage-b", "stage-c|dd-hdr", "final", "tail", "dd-codes+scan",
         "S:wait", "S:hdr+tab", "S:B2+ddhdr", "S:bwr-decode", "S:dd-codes", "S:scans", "S:B3+dma+values", "S:transpose+stores"]
_ser, _dt, _cs, _, _ = W.config("c5")
dp = engine.DevicePipeline(_ser, 23, int(_dt), _cs)
ctx = engine.Context(0)
for var in sys.argv[1:] or ["rand", "ramp"]:
    batch = bench.build_batch(engine, "c5", var, 12500, 128, 0, seed=5)[0]
    ctx.time_launches(3)
    for _ in range(3):
        ctx.unfilter_async(dp, batch)
    torch.cuda.synchronize()
    ms = ctx.last_kernel_ms()
    clk = ctx.phase_clocks(16).astype(np.float64)
    tot = clk.sum()
    print(f"{var}: launch {ms:.4f} ms; per-WG phase share:",
          ", ".join(f"{n} {100 * c / tot:.1f}%" for n, c in zip(NAMES, clk) if c), flush=True)
    del batch
    torch.cuda.empty_cache()
