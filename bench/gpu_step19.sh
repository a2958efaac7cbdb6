set -o pipefail
R=$(pwd)
mkdir -p gpurun_out
export PMD_NO_AUTOBUILD=1
timeout -k 10 300 python bench/conv_bench.py --no-miopen --fp8 > gpurun_out/conv_bench_fp8.log 2>&1 && \
cd /tmp && export TMPDIR=/tmp && \
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof8 -o run -- python $R/bench.py --steps 5 --warmup 3 --dtype fp8 > $R/gpurun_out/prof8.log 2>&1
