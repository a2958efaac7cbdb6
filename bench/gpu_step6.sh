set -o pipefail
mkdir -p gpurun_out
export PMD_NO_AUTOBUILD=1
timeout -k 10 300 python -m pytest tests/test_kernels_gpu.py -x -q > gpurun_out/kern_test.log 2>&1 ; \
PMD_CONV_IMPL=0 timeout -k 10 300 python -m pytest tests/test_kernels_gpu.py -x -q -k "conv_fwd or block" > gpurun_out/kern_test_impl0.log 2>&1 ; \
timeout -k 10 400 python bench/conv_bench.py --batch 256 --iters 10 --impls 0,1 --json gpurun_out/conv_bench.json > gpurun_out/conv_bench.log 2>&1 && \
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --profile gpurun_out/bench_prof.txt > gpurun_out/bench.log 2>&1
