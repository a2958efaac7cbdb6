set -o pipefail
mkdir -p gpurun_out
export PMD_NO_AUTOBUILD=1
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_model_oracle_gpu.py tests/test_distributed_gpu.py tests/test_native_only_gpu.py tests/test_main_e2e_gpu.py > gpurun_out/t6.log 2>&1 &&
AB_ROUNDS=3 bash bench/ab_env.sh "pm1:" "pm0:PMD_PREMASKED=0" > gpurun_out/ab_pm.txt 2>&1
