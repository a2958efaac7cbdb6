# main-stream priority A/B (PMD_MAIN_PRIO=0/1) after the GPU suite
set -o pipefail
mkdir -p gpurun_out
export PMD_NO_AUTOBUILD=1
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 && \
for r in 1 2; do
  for v in 0 1; do
    o=$(PMD_MAIN_PRIO=$v timeout -k 10 200 python bench.py --steps 30 --warmup 10 2>/dev/null | tail -1) || exit 1
    echo "$r prio=$v $(echo "$o" | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')" >> gpurun_out/ab_prio.log
  done
done
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && rm -rf gpurun_out/prof && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run -- python3 bench.py --steps 6 --warmup 4 > gpurun_out/prof.log 2>&1
