# round-5 GPU step 16: BN fold with the prefetching epilogues (apply residual / dot-reduce operands)
set -o pipefail
mkdir -p gpurun_out
export PMD_NO_AUTOBUILD=1
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_bnlin_gpu.py > gpurun_out/t16.log 2>&1 &&
AB_ROUNDS=3 bash bench/ab_env.sh "base:" "fold:PMD_BNFOLD=1" > gpurun_out/ab_fold2.txt 2>&1
