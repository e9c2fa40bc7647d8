#!/bin/bash
# 8-bit ranges whose two windows share the minimum: one-minimum decode (A/B)
set -o pipefail
mkdir -p gpurun_out/is8s
timeout -k 10 300 python -u -m pytest tests/test_gpu_c5tile.py tests/test_gpu_c5_shapes.py -x -q --timeout 120 --timeout-method thread > gpurun_out/is8s/t.log 2>&1 || { tail -30 gpurun_out/is8s/t.log; exit 11; }
tail -1 gpurun_out/is8s/t.log
VARS="ramp rand" bash tools/ab_lib.sh is8s_c5 && VARS="ramp" CFG=c5s bash tools/ab_lib.sh is8s_c5s
