#!/bin/bash
# C5 shapes tests, then the tile kernel on 64 KiB (c5) and 40,000-B (c5s) tiles
set -o pipefail
mkdir -p gpurun_out/r05
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_c5_shapes.py tests/test_gpu_stream.py -m gpu > gpurun_out/r05/t_shapes_${1:-x}.log 2>&1; rc=$?; tail -3 gpurun_out/r05/t_shapes_${1:-x}.log; [ $rc -ne 0 ] && exit $rc
VARS="active rand ramp" ABLS="0" bash tools/c5t_abl.sh ${1:-x}_c5 || exit 1
CFG=c5s VARS="active rand ramp" ABLS="0" bash tools/c5t_abl.sh ${1:-x}_c5s || exit 1
