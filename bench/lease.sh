#!/bin/bash
# One gpurun lease running named measurement presets in order (replaces the per-lease one-off
# scripts of round 5).  Each preset runs under its own time limit through bench/gpu_run.sh,
# which stops at the first crash / timeout.
#   bash bench/lease.sh bench rehearsal fp8 ...        (presets below)
#   BENCH_ARGS="--steps 30 --warmup 10" bash bench/lease.sh bench
set -u
export PMD_NO_AUTOBUILD=1
BA=${BENCH_ARGS:---steps 20 --warmup 5}
specs=()
for p in "$@"; do
  case "$p" in
    gputests)  specs+=("gputests:900:python -u -m pytest tests -m gpu -x -q --timeout 280 --timeout-method thread -p no:cacheprovider") ;;
    bench)     specs+=("bench:240:python bench.py $BA") ;;
    rehearsal) specs+=("rehearsal:240:python bench.py $BA --dp_rehearsal") ;;
    fp8)       specs+=("fp8:240:python bench.py $BA --dtype fp8") ;;
    r152)      specs+=("r152:300:python bench.py $BA --model resnet152") ;;
    stock)     specs+=("stock:400:python bench.py $BA --with_stock") ;;
    long)      specs+=("long:400:python bench.py --steps 300 --warmup 20") ;;
    longfp8)   specs+=("longfp8:400:python bench.py --steps 300 --warmup 20 --dtype fp8") ;;
    prof)      specs+=("prof:300:rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o prof -- python3 bench.py --steps 10 --warmup 5") ;;
    pmc)       specs+=("pmc:600:bash bench/pmc_step.sh") ;;
    contention) specs+=("contention:600:bash bench/contention.sh") ;;
    bytes)     specs+=("bytes:900:bash bench/bytes_budget.sh bf16") ;;
    bytesfp8)  specs+=("bytesfp8:900:bash bench/bytes_budget.sh fp8") ;;
    *) echo "unknown preset $p" >&2; exit 2 ;;
  esac
done
exec bash bench/gpu_run.sh "${specs[@]}"
