# round-5: final bench records (driver command first, then stock comparator, W>1 rehearsal, fp8, ResNet-152)
set -o pipefail
mkdir -p gpurun_out
export PMD_NO_AUTOBUILD=1
O=gpurun_out/bench_final.jsonl
: > $O
timeout -k 10 300 python bench.py 2>gpurun_out/bf_1.err | tail -1 >> $O &&
timeout -k 10 400 python bench.py --with_stock 2>gpurun_out/bf_2.err | tail -1 >> $O &&
timeout -k 10 300 python bench.py --dp_rehearsal 2>gpurun_out/bf_3.err | tail -1 >> $O &&
timeout -k 10 300 python bench.py --dtype fp8 2>gpurun_out/bf_4.err | tail -1 >> $O &&
timeout -k 10 300 python bench.py --model resnet152 2>gpurun_out/bf_5.err | tail -1 >> $O &&
timeout -k 10 300 python bench.py --steps 30 --warmup 10 2>gpurun_out/bf_6.err | tail -1 >> $O
