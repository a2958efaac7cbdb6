set -o pipefail
mkdir -p gpurun_out
export PMD_NO_AUTOBUILD=1
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_bnlin_gpu.py > gpurun_out/t9.log 2>&1 &&
AB_ROUNDS=3 bash bench/ab_env.sh "lin:" "elt:PMD_BNLIN=0" > gpurun_out/ab_lin.txt 2>&1 &&
bash bench/r5_g8.sh
