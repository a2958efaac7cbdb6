# Winograd path: GPU numerics tests + per-layer timing vs implicit GEMM.
set -o pipefail
mkdir -p gpurun_out
export PMD_NO_AUTOBUILD=1
timeout -k 10 300 python -u -m pytest tests/test_winograd_gpu.py -x -v --timeout 120 --timeout-method thread > gpurun_out/wino_tests.log 2>&1 && \
timeout -k 10 300 python bench/winograd_bench.py > gpurun_out/wino_bench.txt 2>&1
