"""bench.py's dense_read_var_host leg alone (GPU box): python tools/dense_leg.py [steps]"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from tiledb_amd import engine  # noqa: E402

ctx = engine.Context(0)
n = int(sys.argv[1]) if len(sys.argv) > 1 else 5
print(json.dumps(bench.dense_var_leg(engine, ctx, n)))
print(json.dumps(bench.dense_var_leg(engine, ctx, n, pinned=True)))
