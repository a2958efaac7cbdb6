# round-5 GPU step 32: after removing the rejected A/B knobs -- wgrad/conv kernel tests + step bench
set -o pipefail
mkdir -p gpurun_out
export PMD_NO_AUTOBUILD=1
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_kernels_gpu.py tests/test_bnlin_gpu.py tests/test_native_only_gpu.py > gpurun_out/t32.log 2>&1 &&
AB_ROUNDS=2 bash bench/ab_env.sh "final:" > gpurun_out/ab32.txt 2>&1
