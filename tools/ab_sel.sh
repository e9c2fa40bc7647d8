#!/bin/bash
# materialize-per-round-count A/B: parity (C5 tile, shapes, C2 tile), then
# same-box bench A/B of HEAD's library against the working tree's
set -o pipefail
mkdir -p gpurun_out/sel
timeout -k 10 300 python -u -m pytest tests/test_gpu_c5tile.py tests/test_gpu_c5_shapes.py tests/test_gpu_c2tile.py -x -q --timeout 120 --timeout-method thread > gpurun_out/sel/t.log 2>&1 || { tail -30 gpurun_out/sel/t.log; exit 11; }
tail -1 gpurun_out/sel/t.log
LIBS="libtiledb_amd_v1.so libtiledb_amd.so" VARS="rand ramp" bash tools/ab_lib.sh sel_c5
