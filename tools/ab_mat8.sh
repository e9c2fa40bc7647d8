#!/bin/bash
# BWR materialization: an all-raw-windows round path (dense-code tiles) A/B
set -o pipefail
mkdir -p gpurun_out/mat8
timeout -k 10 300 python -u -m pytest tests/test_gpu_c5tile.py tests/test_gpu_c5_shapes.py tests/test_gpu_c2tile.py -x -q --timeout 120 --timeout-method thread > gpurun_out/mat8/t.log 2>&1 || { tail -30 gpurun_out/mat8/t.log; exit 11; }
tail -1 gpurun_out/mat8/t.log
VARS="active walk" bash tools/ab_lib.sh mat8_c5 &&
VARS="active" CFG=c5s bash tools/ab_lib.sh mat8_c5s
