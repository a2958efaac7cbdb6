# round-5 GPU step 30: 300-step runs (plain, W>1 rehearsal, fp8) on the final tree
set -o pipefail
mkdir -p gpurun_out
export PMD_NO_AUTOBUILD=1
O=gpurun_out/bench_long.jsonl
: > $O
timeout -k 10 300 python bench.py --steps 300 --warmup 20 2>/dev/null | tail -1 >> $O &&
timeout -k 10 300 python bench.py --steps 300 --warmup 20 --dp_rehearsal 2>/dev/null | tail -1 >> $O &&
timeout -k 10 300 python bench.py --steps 300 --warmup 20 --dtype fp8 2>/dev/null | tail -1 >> $O
