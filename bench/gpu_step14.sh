set -o pipefail
mkdir -p gpurun_out
export PMD_NO_AUTOBUILD=1
timeout -k 10 400 python -m pytest tests/test_kernels_gpu.py -x -q -k conv > gpurun_out/kern_tests.log 2>&1 && \
PMD_CONV_EPI=0 timeout -k 10 300 python bench/conv_bench.py --impls 1,4 --no-miopen > gpurun_out/conv_bench_epi0.log 2>&1 && \
PMD_CONV_EPI=1 timeout -k 10 300 python bench/conv_bench.py --impls 1,4 --no-miopen > gpurun_out/conv_bench_epi1.log 2>&1
