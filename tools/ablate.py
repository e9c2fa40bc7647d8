"""Timing-only ablation of the fused kernel (TDBG_DEBUG_STOP = stop after N stages).
Run on the GPU box (repo root): python tools/ablate.py  -> prints kernel ms per variant."""
import os, subprocess, sys, json
res = {}
for stop in ["1", "2", "3", "0"]:
    for var in ["rand", "ramp"]:
        env = dict(os.environ, TDBG_DEBUG_STOP=stop, TDBG_LIB="libtiledb_amd_exp.so")  # (hooks: experiments library)
        out = subprocess.run([sys.executable, "bench.py", "--steps", "10", "--warmup", "2", "--variants", var,
                              "--no-cpu-baseline"], env=env, capture_output=True, text=True)
        line = [l for l in out.stdout.splitlines() if l.startswith("{")]
        if not line:
            print(stop, var, "FAILED", out.stderr[-2000:]); continue
        d = json.loads(line[-1])
        print(f"stop={stop} {var}: kernel_ms={d['roofline']['kernel_ms']} value={d['value']}", flush=True)
