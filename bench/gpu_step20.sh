set -o pipefail
R=$(pwd)
mkdir -p gpurun_out
export PMD_NO_AUTOBUILD=1
timeout -k 10 300 python -m pytest tests/test_fp8_gpu.py -x -q > gpurun_out/fp8_tests.log 2>&1 && \
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --dtype fp8 > gpurun_out/bench_fp8.log 2>&1 && \
cd /tmp && export TMPDIR=/tmp && \
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof8 -o run -- python $R/bench.py --steps 5 --warmup 3 --dtype fp8 > $R/gpurun_out/prof8.log 2>&1
