set -o pipefail
mkdir -p gpurun_out/r05
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_stream_small.py tests/test_gpu_c5_shapes.py -m gpu > gpurun_out/r05/t_shapes.log 2>&1; rc=$?; tail -3 gpurun_out/r05/t_shapes.log; [ $rc -ne 0 ] && exit $rc
BARGS="--no-cpu-baseline --no-e2e --no-forward --no-others --shard-tiles 0 --c5s-tiles 0" bash tools/profile_all.sh r05a c5 c5s
