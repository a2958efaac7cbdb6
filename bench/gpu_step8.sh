set -o pipefail
mkdir -p gpurun_out
export PMD_NO_AUTOBUILD=1
timeout -k 10 400 python -m pytest tests/ -x -q -m gpu > gpurun_out/gpu_tests.log 2>&1 ; \
timeout -k 10 300 python bench/bn_bench.py > gpurun_out/bn_bench.log 2>&1 ; \
timeout -k 10 300 python bench.py --steps 10 --warmup 3 > gpurun_out/bench.log 2>&1 ; \
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --graph > gpurun_out/bench_graph.log 2>&1
