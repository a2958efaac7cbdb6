# round-5 GPU step 35: LDS-tiled dgrad weight-image transpose -- exactness test, model oracles, step A/B
set -o pipefail
mkdir -p gpurun_out
export PMD_NO_AUTOBUILD=1
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
  tests/test_kernels_gpu.py -k "grouped_weight_images or dgrad" tests/test_bnlin_gpu.py > gpurun_out/wt_tests.txt 2>&1 &&
AB_ROUNDS=3 bash bench/ab_so.sh base tile tile base > gpurun_out/ab_wtile.txt 2>&1
