# round-5 GPU step 37: one tile walk writes both bf16 weight images (mode 3) -- tests, step A/B, kernel trace
set -o pipefail
mkdir -p gpurun_out
export PMD_NO_AUTOBUILD=1 PMD_ALLOW_VARIANT=1
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
  tests/test_kernels_gpu.py -k "weight_images or dgrad" tests/test_fp8_gpu.py > gpurun_out/wtf_tests.txt 2>&1 &&
bash bench/ab_so.sh tile8 fused fused tile8 > gpurun_out/ab_wfused.txt 2>&1 &&
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" &&
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/wt_fused -o run -- python3 bench.py --steps 12 --warmup 6 > gpurun_out/wt_fused.log 2>&1
