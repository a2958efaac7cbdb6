export PMD_NO_AUTOBUILD=1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
bash bench/gpu_run.sh \
 "s1tests:300:python -u -m pytest tests/test_kernels_gpu.py -k \"conv1x1_stream or wgrad\" -q --timeout 120 --timeout-method thread" \
 "epi1:200:python bench/dgrad_epi_bench.py --iters 20 --s1 1" \
 "epi1_64:200:python bench/dgrad_epi_bench.py --iters 20 --s1 1 --s1bn 64" \
 "fwd0:200:python bench/fwd1x1_bench.py" \
 "fwd2:200:python bench/fwd1x1_bench.py --s1 2" \
 "r50s1:200:PMD_CONV1X1=1 python bench.py --steps 30 --warmup 10" \
 "r50s2:200:PMD_CONV1X1=2 python bench.py --steps 30 --warmup 10" \
 "r50:200:python bench.py --steps 30 --warmup 10" \
 "prof_reh:300:rocprofv3 --kernel-trace --stats -d gpurun_out/prof_reh -o run -- python3 bench.py --steps 10 --warmup 5 --dp_rehearsal" \
 "prof_reh_c10d:300:rocprofv3 --kernel-trace --stats -d gpurun_out/prof_reh_c10d -o run -- python3 bench.py --steps 10 --warmup 5 --dp_rehearsal --comm c10d" \
 "prof_plain:300:rocprofv3 --kernel-trace --stats -d gpurun_out/prof_plain -o run -- python3 bench.py --steps 10 --warmup 5" \
 "tests2:600:python -u -m pytest tests/test_fp8_gpu.py tests/test_multirank_gpu.py -x -q --timeout 300 --timeout-method thread"
bash bench/gpu_run.sh \
 "cprof_reh:300:python -m cProfile -s tottime bench.py --steps 20 --warmup 5 --dp_rehearsal" \
 "cprof_plain:300:python -m cProfile -s tottime bench.py --steps 20 --warmup 5"
bash bench/gpu_run.sh \
 "prof_w2q:400:rocprofv3 --kernel-trace -d gpurun_out/prof_w2q -o run -- python3 bench.py --gpus 2 --backend gloo --same_device --syncbn_comm xgmi --steps 4 --warmup 2" \
 "reh_dbg:300:PMD_SYNC_DEBUG=1 python bench.py --steps 3 --warmup 2 --dp_rehearsal"
bash bench/gpu_run.sh \
 "reh_q8:200:GPU_MAX_HW_QUEUES=8 python bench.py --steps 30 --warmup 10 --dp_rehearsal" \
 "reh_c10d_q8:200:GPU_MAX_HW_QUEUES=8 python bench.py --steps 30 --warmup 10 --dp_rehearsal --comm c10d" \
 "plain_q8:200:GPU_MAX_HW_QUEUES=8 python bench.py --steps 30 --warmup 10" \
 "reh_noov:200:PMD_SYNCBN_OVERLAP=0 python bench.py --steps 30 --warmup 10 --dp_rehearsal"
