export PMD_NO_AUTOBUILD=1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
bash bench/gpu_run.sh \
 "s1tests:300:python -u -m pytest tests/test_kernels_gpu.py -k \"conv1x1_stream\" -q --timeout 120 --timeout-method thread" \
 "f8tests:400:python -u -m pytest tests/test_fp8_gpu.py -x -q --timeout 200 --timeout-method thread" \
 "protest:200:python -u -m pytest tests/test_kernels_gpu.py -k bn_prologue -q --timeout 100 --timeout-method thread" \
 "pro:200:python bench/bn_prologue_bench.py" \
 "r50:200:python bench.py --steps 30 --warmup 10" \
 "r50_f8:200:python bench.py --steps 30 --warmup 10 --dtype fp8" \
 "reh:200:python bench.py --steps 30 --warmup 10 --dp_rehearsal" \
 "reh_c10d:200:python bench.py --steps 30 --warmup 10 --dp_rehearsal --comm c10d" \
 "r152:300:python bench.py --steps 20 --warmup 8 --model resnet152" \
 "r152_reh:300:python bench.py --steps 20 --warmup 8 --model resnet152 --dp_rehearsal" \
 "hp_plain:200:python bench.py --steps 10 --warmup 5 --host_profile gpurun_out/hostprof_plain.txt" \
 "hp_reh:200:python bench.py --steps 10 --warmup 5 --dp_rehearsal --host_profile gpurun_out/hostprof_reh.txt" \
 "prof_reh:300:rocprofv3 --kernel-trace --stats -d gpurun_out/prof_reh4 -o run -- python3 bench.py --steps 10 --warmup 5 --dp_rehearsal" \
 "prof_plain:300:rocprofv3 --kernel-trace --stats -d gpurun_out/prof_plain4 -o run -- python3 bench.py --steps 10 --warmup 5" \
 "pmc_f8:500:bash bench/pmc_step.sh gpurun_out/pmc_fp8_r04 -- python3 bench.py --steps 2 --warmup 1 --dtype fp8"
