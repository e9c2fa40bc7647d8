#!/bin/bash
# materialize-per-round-count A/B: parity (C5 tile, shapes, C2 tile), then
# same-box bench A/B of HEAD's library against the working tree's
set -o pipefail
mkdir -p gpurun_out/rawf
timeout -k 10 300 python -u -m pytest tests/test_gpu_c5tile.py tests/test_gpu_c5_shapes.py tests/test_gpu_c2tile.py -x -q --timeout 120 --timeout-method thread > gpurun_out/rawf/t.log 2>&1 || { tail -30 gpurun_out/rawf/t.log; exit 11; }
tail -1 gpurun_out/rawf/t.log
VARS="rand ramp" bash tools/ab_lib.sh rawf_c5 && VARS="rand" CFG=c5s bash tools/ab_lib.sh rawf_c5s
