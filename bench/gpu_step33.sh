set -o pipefail
mkdir -p gpurun_out
export PMD_NO_AUTOBUILD=1
timeout -k 10 500 python -m pytest tests/test_kernels_gpu.py -x -q -k "pool or resnet50" > gpurun_out/gpu_tests.log 2>&1 && \
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/bench.log 2>&1
