# round-5 GPU step 19: unpadded XOR-swizzled dgrad C staging (PMD_EPI_X): kernel tests, A/B vs the padded layout
set -o pipefail
mkdir -p gpurun_out
export PMD_NO_AUTOBUILD=1
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_kernels_gpu.py tests/test_bnlin_gpu.py tests/test_model_oracle_gpu.py > gpurun_out/t19.log 2>&1 &&
bash bench/ab_so.sh x1 x0 > gpurun_out/ab_x.txt 2>&1
