# round-5 GPU step 36: tiled fp8 weight quant -- exactness + fp8 tests, fp8 step A/B,
# and kernel traces of the weight-prep kernels before / after the LDS-tiled transposes
set -o pipefail
mkdir -p gpurun_out
export PMD_NO_AUTOBUILD=1 PMD_ALLOW_VARIANT=1
SO=pytorch_multiprocessing_distributed_amd/_C.cpython-310-x86_64-linux-gnu.so
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
  tests/test_kernels_gpu.py -k "weight_images" tests/test_fp8_gpu.py > gpurun_out/wt8_tests.txt 2>&1 &&
AB_ARGS="--dtype fp8" bash bench/ab_so.sh tile tile8 tile8 tile > gpurun_out/ab_wtile8.txt 2>&1 &&
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" &&
for v in base tile8; do
  cp abso/so_$v.so $SO &&
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/wt_$v -o run -- python3 bench.py --steps 12 --warmup 6 > gpurun_out/wt_$v.log 2>&1 || exit 1
done
cp abso/so_tile8.so $SO
