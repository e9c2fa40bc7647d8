"""Phase clocks of the one-workgroup-per-tile C5 kernel (tdbg_c5tile.hip) on
the bench's 100,000-tile workload.  Run on the GPU box:
  TDBG_PROF=1 python tools/c5t_prof.py rand ramp"""
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

NAMES = (["dma-wait", "parse", "setup", "w0-decode+st", "w1-decode+st", "w15-decode+st", "wg-total"]
         if "active" not in sys.argv else
         ["dma-wait", "parse", "codes+scan", "B3+fold+vwrite", "B4", "transp+stores", "w15 codes..end"])
_ser, _dt, _cs, _, _ = W.config("c5")
dp = engine.DevicePipeline(_ser, 23, int(_dt), _cs)
ctx = engine.Context(0)
for var in sys.argv[1:] or ["rand", "ramp"]:
    batch = bench.build_batch(engine, "c5", var, 100000, 128, 0, seed=5)[0]
    ctx.time_launches(3)
    for _ in range(3):
        ctx.unfilter_async(dp, batch)
    torch.cuda.synchronize()
    ms = ctx.last_kernel_ms()
    clk = ctx.phase_clocks(16).astype(np.float64)[8:] / 1024.0
    print(f"{var}: launch {ms:.4f} ms; mean s_memtime ticks per workgroup (100 MHz):",
          ", ".join(f"{n} {c:.0f}" for n, c in zip(NAMES, clk)), flush=True)
    del batch
    torch.cuda.empty_cache()
