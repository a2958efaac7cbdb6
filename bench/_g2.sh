export PMD_NO_AUTOBUILD=1
bash bench/gpu_run.sh \
 "tests:900:python -u -m pytest tests/test_kernels_gpu.py tests/test_fp8_gpu.py tests/test_multirank_gpu.py -x -q --timeout 300 --timeout-method thread" \
 "r50:200:python bench.py --steps 30 --warmup 10" \
 "r50reh:200:python bench.py --steps 30 --warmup 10 --dp_rehearsal" \
 "r50reh_c10d:200:python bench.py --steps 30 --warmup 10 --dp_rehearsal --comm c10d" \
 "r152:300:python bench.py --model resnet152 --steps 20 --warmup 10" \
 "r152reh:300:python bench.py --model resnet152 --steps 20 --warmup 10 --dp_rehearsal"
