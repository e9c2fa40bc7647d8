"""Diagnostics: run one C1 / C5 batch through the engine in a child process per
mode (no view kernel / view kernel only / full), each under its own timeout."""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CHILD = r'''
import sys, numpy as np, torch
sys.path.insert(0, %r)
from tests.cases import config_cases
from oracle import oracle as O
from tiledb_amd import engine
case = [c for c in config_cases(4) if c.name == sys.argv[1]][0]
op = O.OraclePipeline(case.serialized, case.version, int(case.dtype), case.cell_size)
enc = [np.frombuffer(op.filter_tile(t), dtype=np.uint8) for t in case.tiles]
dp = engine.DevicePipeline(case.serialized, case.version, int(case.dtype), case.cell_size)
ctx = engine.Context(0)
batch = engine.TileBatch.from_host(enc, [t.size for t in case.tiles])
import ctypes
from tiledb_amd._native import lib
q = (ctypes.c_uint32 * 4)()
lib.tdbg_debug_queue_counts(ctx.h, q)
print("queues before", list(q), flush=True)
print("launching", flush=True)
ctx.unfilter_async(dp, batch)
torch.cuda.synchronize()
lib.tdbg_debug_queue_counts(ctx.h, q)
print("queues after", list(q), flush=True)
print("synced; status", batch.d_status.cpu().numpy(), flush=True)
out = batch.outputs_host()
ok = all(np.array_equal(out[int(batch.out_off[i]):int(batch.out_off[i]) + t.size], t) for i, t in enumerate(case.tiles))
print("match", ok, flush=True)
''' % ROOT
for name in sys.argv[1:] or ["C1_ramp"]:
    F = {"TDBG_VIEW": "1"}
    for mode, env in (("aligned view+fused-on-nothing", dict(F, TDBG_DEBUG_FUSED_EMPTY="1",
                                                             TDBG_DEBUG_SKIP_FIXUP="1")),
                      ("aligned full", dict(F)), ("aligned full again", dict(F))):
        e = dict(os.environ, **env)
        try:
            r = subprocess.run([sys.executable, "-c", CHILD, name], env=e, capture_output=True, text=True,
                               timeout=40)
            print(name, mode, "rc", r.returncode, r.stdout.strip().replace("\n", " | "), r.stderr[:1200],
                  flush=True)
            if r.returncode != 0:
                sys.exit(1)
        except subprocess.TimeoutExpired as ex:
            print(name, mode, "TIMEOUT", (ex.stdout or b"")[-400:], flush=True)
            err = (ex.stderr or b"").decode(errors="replace").splitlines()
            print("\n".join(err[-60:]), flush=True)
            sys.exit(2)
