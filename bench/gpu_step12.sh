set -o pipefail
mkdir -p gpurun_out
export PMD_NO_AUTOBUILD=1
timeout -k 10 400 python -m pytest tests/test_kernels_gpu.py -x -q -k "conv" > gpurun_out/conv_tests.log 2>&1 && \
timeout -k 10 500 python bench/conv_bench.py --impls 1,2,3,4 --no-miopen > gpurun_out/conv_bench_impls.log 2>&1 && \
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/bench.log 2>&1
