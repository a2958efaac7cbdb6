set -o pipefail
mkdir -p gpurun_out
export PMD_NO_AUTOBUILD=1
timeout -k 10 400 python bench.py --model resnet152 --steps 10 --warmup 3 > gpurun_out/bench_r152.log 2>&1
