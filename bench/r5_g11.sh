# round-5 GPU step 11: BN fold (statistics-only conv3 + BN-apply epilogue, dot-only reduce):
# bnlin/fold tests, then the step A/B
set -o pipefail
mkdir -p gpurun_out
export PMD_NO_AUTOBUILD=1
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_bnlin_gpu.py > gpurun_out/t11.log 2>&1 &&
AB_ROUNDS=3 bash bench/ab_env.sh "fold:" "lin:PMD_BNFOLD=0" "folda:PMD_BNLIN=all" "elt:PMD_BNLIN=0" > gpurun_out/ab_fold.txt 2>&1
