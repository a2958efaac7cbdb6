set -o pipefail
mkdir -p gpurun_out
export PMD_NO_AUTOBUILD=1
timeout -k 10 400 python -m pytest tests/test_kernels_gpu.py -x -q -k "conv" > gpurun_out/kern_tests.log 2>&1 && \
timeout -k 10 400 python bench/conv_bench.py --no-miopen --impls 1,4,6 > gpurun_out/conv_bench_mf32.log 2>&1
