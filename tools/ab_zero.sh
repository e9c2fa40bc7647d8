set -o pipefail
mkdir -p gpurun_out/zero
timeout -k 10 300 python -u -m pytest tests/test_gpu_c5tile.py tests/test_gpu_c5_shapes.py -x -q --timeout 120 --timeout-method thread > gpurun_out/zero/t.log 2>&1 || { tail -30 gpurun_out/zero/t.log; exit 11; }
tail -1 gpurun_out/zero/t.log
VARS="active" bash tools/ab_lib.sh zero_c5 && VARS="active" CFG=c5s bash tools/ab_lib.sh zero_c5s && VARS="active" CFG=c5big bash tools/ab_lib.sh zero_c5big
