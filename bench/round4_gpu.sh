# The round-4 GPU measurements in one place (run through gpurun from the repo root; every step
# under its own time limit via bench/gpu_run.sh).  Results land in gpurun_out/<name>.log;
# profiles/ holds the committed summaries (rehearsal_r04.txt, queues_r04.txt, bench_r04_*.jsonl,
# pmc_r50_*_r04.txt, conv1x1_stream_r04.txt, bn_prologue_r04.txt).
#   bash bench/round4_gpu.sh [bench|rehearsal|queues|pmc|kernels|tests]
export PMD_NO_AUTOBUILD=1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
case "${1:-bench}" in
  bench) bash bench/gpu_run.sh \
    "fresh:300:python bench.py" \
    "r50:200:python bench.py --steps 30 --warmup 10" \
    "f8:200:python bench.py --steps 30 --warmup 10 --dtype fp8" \
    "r152:300:python bench.py --steps 20 --warmup 8 --model resnet152" ;;
  rehearsal) bash bench/gpu_run.sh \
    "r50:200:python bench.py --steps 30 --warmup 10" \
    "reh:200:python bench.py --steps 30 --warmup 10 --dp_rehearsal" \
    "reh_c10d:200:python bench.py --steps 30 --warmup 10 --dp_rehearsal --comm c10d" \
    "r152:300:python bench.py --steps 20 --warmup 8 --model resnet152" \
    "r152_reh:300:python bench.py --steps 20 --warmup 8 --model resnet152 --dp_rehearsal" \
    "hp_reh:200:python bench.py --steps 10 --warmup 5 --dp_rehearsal --host_profile gpurun_out/hostprof_reh.txt" ;;
  queues) bash bench/gpu_run.sh \
    "prof_reh:300:rocprofv3 --kernel-trace -d gpurun_out/prof_reh -o run -- python3 bench.py --steps 10 --warmup 5 --dp_rehearsal" \
    "prof_w2:240:rocprofv3 --kernel-trace -d gpurun_out/prof_w2 -o run_%pid% -- python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29534 bench.py --gpus 2 --same_device --backend gloo --syncbn_comm xgmi --steps 3 --warmup 2 --batch 32"
    # then: python bench/queue_map.py gpurun_out/prof_reh/run_results.db --steps-only (and each prof_w2/*.db)
    ;;
  pmc) bash bench/gpu_run.sh \
    "pmc_bf16:500:bash bench/pmc_step.sh gpurun_out/pmc_r04" \
    "pmc_f8:500:bash bench/pmc_step.sh gpurun_out/pmc_fp8_r04 -- python3 bench.py --steps 2 --warmup 1 --dtype fp8"
    # then: python bench/pmc_summary.py gpurun_out/pmc_r04
    ;;
  kernels) bash bench/gpu_run.sh \
    "epi:200:python bench/dgrad_epi_bench.py --iters 20" \
    "epi_s1:200:python bench/dgrad_epi_bench.py --iters 20 --s1 1" \
    "fwd1x1:200:python bench/fwd1x1_bench.py" \
    "fwd1x1_s1:200:python bench/fwd1x1_bench.py --s1 2" \
    "pro:200:python bench/bn_prologue_bench.py" ;;
  tests) bash bench/gpu_run.sh \
    "gputests:900:python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread" ;;
esac
