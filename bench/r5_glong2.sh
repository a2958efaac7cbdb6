# round-5: 300-step runs on the final tree (bf16, W>1 rehearsal, fp8)
set -o pipefail
mkdir -p gpurun_out
export PMD_NO_AUTOBUILD=1
O=gpurun_out/bench_long2.jsonl
: > $O
timeout -k 10 300 python bench.py --steps 300 --warmup 10 2>gpurun_out/bl_1.err | tail -1 >> $O &&
timeout -k 10 300 python bench.py --steps 300 --warmup 10 --dp_rehearsal 2>gpurun_out/bl_2.err | tail -1 >> $O &&
timeout -k 10 300 python bench.py --steps 300 --warmup 10 --dtype fp8 2>gpurun_out/bl_3.err | tail -1 >> $O
