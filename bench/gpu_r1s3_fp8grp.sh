# grouped fp8 weight quantisation: fp8 tests, full GPU suite, fp8 + bf16 bench
set -o pipefail
mkdir -p gpurun_out
export PMD_NO_AUTOBUILD=1
timeout -k 10 300 python -u -m pytest tests/test_fp8_gpu.py -x -v --timeout 120 --timeout-method thread > gpurun_out/fp8_tests.log 2>&1 && \
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 && \
timeout -k 10 300 python bench.py --dtype fp8 --steps 30 --warmup 10 > gpurun_out/bench_fp8.log 2>&1 && \
timeout -k 10 300 python bench.py --steps 30 --warmup 10 > gpurun_out/bench_r50.log 2>&1
