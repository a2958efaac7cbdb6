# Final verification of the committed tree: smoke, GPU suite, R50 bench, steady-state trace, R152/fp8 benches.
set -o pipefail
mkdir -p gpurun_out
export PMD_NO_AUTOBUILD=1
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 && \
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 && \
timeout -k 10 300 python bench.py --steps 30 --warmup 10 > gpurun_out/bench_r50.log 2>&1 && \
timeout -k 10 300 python bench.py --model resnet152 --steps 20 --warmup 5 > gpurun_out/bench_r152.log 2>&1 && \
timeout -k 10 300 python bench.py --dtype fp8 --steps 30 --warmup 10 > gpurun_out/bench_fp8.log 2>&1 && \
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && rm -rf gpurun_out/prof && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run -- python3 bench.py --steps 6 --warmup 4 > gpurun_out/prof.log 2>&1
