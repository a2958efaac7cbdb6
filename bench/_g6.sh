export PMD_NO_AUTOBUILD=1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
bash bench/gpu_run.sh \
 "s1tests:300:python -u -m pytest tests/test_kernels_gpu.py -k \"conv1x1_stream\" -q --timeout 120 --timeout-method thread" \
 "f8tests:400:python -u -m pytest tests/test_fp8_gpu.py -x -q --timeout 200 --timeout-method thread" \
 "r50:200:python bench.py --steps 30 --warmup 10" \
 "r50_f8:200:python bench.py --steps 30 --warmup 10 --dtype fp8" \
 "reh:200:python bench.py --steps 30 --warmup 10 --dp_rehearsal" \
 "reh_prio:200:PMD_STREAM_PRIO=1 python bench.py --steps 30 --warmup 10 --dp_rehearsal" \
 "reh_q8:200:GPU_MAX_HW_QUEUES=8 python bench.py --steps 30 --warmup 10 --dp_rehearsal" \
 "reh_c10d:200:python bench.py --steps 30 --warmup 10 --dp_rehearsal --comm c10d" \
 "reh_c10d_prio:200:PMD_STREAM_PRIO=1 python bench.py --steps 30 --warmup 10 --dp_rehearsal --comm c10d" \
 "r50_prio:200:PMD_STREAM_PRIO=1 python bench.py --steps 30 --warmup 10"
