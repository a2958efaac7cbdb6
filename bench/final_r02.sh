# Round-2 end-of-round measurement set (one gpurun call): full GPU suite, smoke,
# bf16/fp8/R152 benches, rocprofv3 kernel stats of the bf16 step, PMC counters.
set -o pipefail
export PMD_NO_AUTOBUILD=1
bash bench/gpu_run.sh \
  "gpu:900:python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread" \
  "smoke:200:python -c 'import __graft_entry__ as g; g.smoke(); print(\"smoke ok\")'" \
  "b50:300:python bench.py --steps 30 --warmup 10" \
  "bfp8:300:python bench.py --steps 30 --warmup 10 --dtype fp8" \
  "b152:300:python bench.py --steps 20 --warmup 5 --model resnet152" \
  "prof:300:cd /tmp && export TMPDIR=/tmp && cd \$GRAFT_REPO_ROOT && rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run -- python3 bench.py --steps 8 --warmup 3" \
  "pmc:500:bash bench/pmc_step.sh"
