export PMD_NO_AUTOBUILD=1
bash bench/gpu_run.sh \
 "s1tests:300:python -u -m pytest tests/test_kernels_gpu.py -k conv1x1_stream -x -q --timeout 120 --timeout-method thread" \
 "epi0:200:python bench/dgrad_epi_bench.py --iters 20" \
 "epi1:200:python bench/dgrad_epi_bench.py --iters 20 --s1 1" \
 "epi1_64:200:python bench/dgrad_epi_bench.py --iters 20 --s1 1 --s1bn 64" \
 "r50:200:python bench.py --steps 30 --warmup 10" \
 "r50s1:200:PMD_CONV1X1=1 python bench.py --steps 30 --warmup 10" \
 "r50s2:200:PMD_CONV1X1=2 python bench.py --steps 30 --warmup 10" \
 "tests:900:python -u -m pytest tests/test_kernels_gpu.py tests/test_fp8_gpu.py tests/test_multirank_gpu.py -x -q --timeout 300 --timeout-method thread" \
 "r50reh:200:python bench.py --steps 30 --warmup 10 --dp_rehearsal" \
 "r50reh_c10d:200:python bench.py --steps 30 --warmup 10 --dp_rehearsal --comm c10d" \
 "r152:300:python bench.py --model resnet152 --steps 20 --warmup 10" \
 "r152reh:300:python bench.py --model resnet152 --steps 20 --warmup 10 --dp_rehearsal"
