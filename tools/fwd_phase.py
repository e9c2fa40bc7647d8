"""Per-phase cycle breakdown of the LDS-resident C5 forward kernel
(tdbg_forward_stream.hip) on the bench's C5 tiles.
Run on the GPU box:  python tools/fwd_phase.py [variant ...]"""
import os, sys
os.environ.setdefault("TDBG_PROF", "1")
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np
import torch
import workloads as W
from tiledb_amd import engine

NAMES = ["loads+transposes", "bitsize+B1", "dd-out+B2", "bwr-windows+B3", "scan+headers+B4/B5",
         "compress+B6", "store"]
ser, dt, cs, _, _ = W.config("c5")
dp = engine.DevicePipeline(ser, 23, int(dt), cs)
ctx = engine.Context(0)
for var in sys.argv[1:] or ["active", "rand"]:
    rng = np.random.default_rng(5)
    vals = [W.c5_values(var, k, rng) for k in range(128)]
    fb = ctx.filter_batch(dp, [vals[i % 128] for i in range(12500)])
    for _ in range(3):
        ctx.filter_async(dp, fb, stream=torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    clk = ctx.phase_clocks(16).astype(np.float64)[:7]
    tot = clk.sum()
    print(f"{var}: per-WG phase share:", ", ".join(f"{n} {100 * c / tot:.1f}%" for n, c in zip(NAMES, clk)),
          f"(total {tot / 512 / 1e3:.1f} kcycles per WG)", flush=True)
    del fb
    torch.cuda.empty_cache()
