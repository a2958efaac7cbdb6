set -o pipefail
mkdir -p gpurun_out
export PMD_NO_AUTOBUILD=1
timeout -k 10 400 python -m pytest tests/ -x -q -m gpu > gpurun_out/gpu_tests.log 2>&1 ; \
timeout -k 10 300 python bench/conv_bench.py --batch 256 --iters 10 --impls 1 --no-miopen --json gpurun_out/conv_bench.json > gpurun_out/conv_bench.log 2>&1 && \
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --profile gpurun_out/bench_prof.txt > gpurun_out/bench.log 2>&1
