set -o pipefail
mkdir -p gpurun_out
export PMD_NO_AUTOBUILD=1
timeout -k 10 300 python -m pytest tests/test_fp8_gpu.py -x -q > gpurun_out/fp8_tests.log 2>&1 ; \
timeout -k 10 300 python bench/dbg_fp8c.py > gpurun_out/dbg_fp8c.log 2>&1 && \
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --dtype fp8 > gpurun_out/bench_fp8.log 2>&1
