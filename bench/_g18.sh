export PMD_NO_AUTOBUILD=1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
bash bench/gpu_run.sh \
 "f8fwdt:300:python -u -m pytest tests/test_fp8_gpu.py -x -q -k conv_fp8_fwd --timeout 100 --timeout-method thread" \
 "f8a0:200:python bench.py --steps 30 --warmup 10 --dtype fp8" \
 "f8a1:200:PMD_FP8_FWD_IMPL=1 python bench.py --steps 30 --warmup 10 --dtype fp8" \
 "f8b0:200:python bench.py --steps 30 --warmup 10 --dtype fp8" \
 "f8b1:200:PMD_FP8_FWD_IMPL=1 python bench.py --steps 30 --warmup 10 --dtype fp8" \
 "f8tall:300:PMD_FP8_FWD_IMPL=1 python -u -m pytest tests/test_fp8_gpu.py -x -q --timeout 200 --timeout-method thread"
