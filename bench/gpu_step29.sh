set -o pipefail
mkdir -p gpurun_out
export PMD_NO_AUTOBUILD=1
for B in 512 1024 2048; do
PMD_WGRAD_BLOCKS=$B timeout -k 10 300 python bench/conv_bench.py --no-miopen > gpurun_out/conv_bench_wg$B.log 2>&1 || exit 1
done
