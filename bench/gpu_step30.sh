set -o pipefail
mkdir -p gpurun_out
export PMD_NO_AUTOBUILD=1
PMD_WGRAD_BLOCKS_R1=256 timeout -k 10 300 python bench/conv_bench.py --no-miopen --only _R1_ > gpurun_out/conv_bench_wg256.log 2>&1 && \
timeout -k 10 400 python -m pytest tests/test_kernels_gpu.py -x -q -k "conv or wgrad" > gpurun_out/kern_tests.log 2>&1 && \
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/bench.log 2>&1
