set -o pipefail
mkdir -p gpurun_out
export PMD_NO_AUTOBUILD=1
timeout -k 10 300 python -m pytest tests/test_kernels_gpu.py -x -q -k "bn or bwd" > gpurun_out/gpu_tests_bn.log 2>&1 && \
timeout -k 10 300 python bench/bn_bench.py > gpurun_out/bn_bench2.log 2>&1 && \
timeout -k 10 300 python bench/dbg_r50.py > gpurun_out/dbg_r50.log 2>&1
