set -o pipefail
mkdir -p gpurun_out
export PMD_NO_AUTOBUILD=1
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_bnlin_gpu.py > gpurun_out/t10.log 2>&1 &&
AB_ROUNDS=3 bash bench/ab_env.sh "lin:" "lin3:PMD_BNLIN_MIN=40000000" "lina:PMD_BNLIN=all" "elt:PMD_BNLIN=0" > gpurun_out/ab_lin2.txt 2>&1
