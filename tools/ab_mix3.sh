#!/bin/bash
# mixed raw/8-bit ranges through the one-read path: parity of the C5 tile
# tests, then a same-box A/B: _v1 = HEAD, _sel = branch-free 8-bit select,
# libtiledb_amd.so = select + mixed ranges
set -o pipefail
mkdir -p gpurun_out/mix3
timeout -k 10 300 python -u -m pytest tests/test_gpu_c5tile.py tests/test_gpu_c5_shapes.py -x -q --timeout 120 --timeout-method thread > gpurun_out/mix3/t.log 2>&1 || { tail -30 gpurun_out/mix3/t.log; exit 11; }
tail -1 gpurun_out/mix3/t.log
LIBS="libtiledb_amd_base.so libtiledb_amd.so" VARS="ramp rand" bash tools/ab_lib.sh mix3_c5 && LIBS="libtiledb_amd_base.so libtiledb_amd.so" VARS="ramp" CFG=c5s bash tools/ab_lib.sh mix3_c5s
