#!/bin/bash
# round 5 GPU check: every -m gpu test, then the C5 variants A/B (product vs
# the persistent kernels) and the one-workgroup-per-tile kernel's phase clocks
set -o pipefail
mkdir -p gpurun_out/r05
timeout -k 10 900 python -u -m pytest -x -q --timeout 180 --timeout-method thread tests -m gpu > gpurun_out/r05/t_gpu_${1:-x}.log 2>&1
rc=$?; tail -4 gpurun_out/r05/t_gpu_${1:-x}.log; [ $rc -ne 0 ] && exit $rc
VARS="active rand ramp" ABLS="old 0" bash tools/c5t_abl.sh ${1:-x} || exit 1
timeout -k 10 200 python tools/c5t_prof.py active rand
