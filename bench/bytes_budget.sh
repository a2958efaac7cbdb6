#!/bin/bash
# Bytes budget of one ResNet-50 step for a dtype: rocprofv3 PMC passes (bench/pmc_step.sh) + a
# kernel trace of the two-stream step, then bench/bytes_budget.py.
#   bash bench/bytes_budget.sh bf16|fp8 [outdir]
set -o pipefail
dt=${1:-bf16}
out=${2:-gpurun_out/bytes_$dt}
mkdir -p "$out"
root=$(pwd)
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$root}"
export PMD_NO_AUTOBUILD=1
bash bench/pmc_step.sh "$out/pmc" -- python3 bench.py --steps 2 --warmup 1 --dtype "$dt" || exit 1
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d "$out/trace" -o run -- \
  python3 bench.py --steps 10 --warmup 5 --dtype "$dt" > "$out/trace.log" 2>&1 || exit 1
python bench/bytes_budget.py "$out/pmc" "$(find "$out/trace" -name '*kernel_trace.csv' | head -1)" \
  --warmup 5 --steps 10 --title "ResNet-50 bs256 $dt, round-6 tree"
