set -o pipefail
mkdir -p gpurun_out
export PMD_NO_AUTOBUILD=1
timeout -k 10 300 python -m pytest tests/test_kernels_gpu.py -x -q > gpurun_out/kern_test.log 2>&1 && \
timeout -k 10 400 python bench.py --steps 10 --warmup 3 --profile gpurun_out/bench_prof.txt > gpurun_out/bench.log 2>&1
