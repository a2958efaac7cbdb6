# BASELINE configs 2/4/5 on one GPU with the current tree: R50 bf16, R152 bf16, R50 fp8 (+ steady-state trace of R50)
set -o pipefail
mkdir -p gpurun_out
export PMD_NO_AUTOBUILD=1
timeout -k 10 300 python bench.py --steps 30 --warmup 10 > gpurun_out/bench_r50.log 2>&1 && \
timeout -k 10 300 python bench.py --model resnet152 --steps 20 --warmup 5 > gpurun_out/bench_r152.log 2>&1 && \
timeout -k 10 300 python bench.py --dtype fp8 --steps 30 --warmup 10 > gpurun_out/bench_fp8.log 2>&1 && \
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
