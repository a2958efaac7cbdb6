# s2d stem: GPU numerics tests, then the full GPU suite, then A/B bench (PMD_STEM_S2D on/off).
set -o pipefail
mkdir -p gpurun_out
export PMD_NO_AUTOBUILD=1
timeout -k 10 300 python -u -m pytest tests/test_stem_s2d_gpu.py -x -v --timeout 120 --timeout-method thread > gpurun_out/s2d_tests.log 2>&1 && \
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 && \
for r in 1 2; do
  for v in 0 1; do
    o=$(PMD_STEM_S2D=$v timeout -k 10 200 python bench.py --steps 30 --warmup 10 2>/dev/null | tail -1) || exit 1
    echo "$r s2d=$v $(echo "$o" | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')" >> gpurun_out/ab_s2d.log
  done
done
