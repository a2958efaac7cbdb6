#!/bin/bash
# Contention attribution of the two-stream step: kernel traces of the same bench run with the
# weight gradients on the side stream (two_stream) and on the main stream (one_stream), then
# bench/contention.py.   bash bench/contention.sh [outdir] [extra bench.py args]
set -o pipefail
out=${1:-gpurun_out/contention}; shift || true
mkdir -p "$out"
root=$(pwd)
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$root}"
export PMD_NO_AUTOBUILD=1
for m in two_stream one_stream; do
  timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d "$out/$m" -o run -- \
    python3 bench.py --steps 12 --warmup 5 --step_mode $m "$@" > "$out/$m.log" 2>&1 || exit 1
done
python bench/contention.py "$out/two_stream" "$out/one_stream" --step 8
