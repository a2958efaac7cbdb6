set -o pipefail
mkdir -p gpurun_out
export PMD_NO_AUTOBUILD=1
timeout -k 10 300 python bench/conv_bench.py --no-miopen --bnred > gpurun_out/conv_bench_bnred.log 2>&1
