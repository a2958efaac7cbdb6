set -o pipefail
R=$(pwd)
mkdir -p gpurun_out
export PMD_NO_AUTOBUILD=1
timeout -k 10 400 python -m pytest tests/test_kernels_gpu.py -x -q > gpurun_out/kern_tests.log 2>&1 && \
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/bench.log 2>&1 && \
timeout -k 10 300 python bench/conv_bench.py --no-miopen > gpurun_out/conv_bench_v7.log 2>&1
