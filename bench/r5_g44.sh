# round-5 GPU step 44: weight gradients wait on their dY kernel's completion event (PMD_FORK_ELEMT) --
# tests, then the step A/B against the fork markers
set -o pipefail
mkdir -p gpurun_out
export PMD_NO_AUTOBUILD=1
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_stream_events_gpu.py > gpurun_out/sev2_tests.txt 2>&1 &&
PMD_FORK_ELEMT=1 timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_model_oracle_gpu.py tests/test_fp8_gpu.py tests/test_distributed_gpu.py tests/test_bnlin_gpu.py > gpurun_out/sev2_oracle.txt 2>&1 &&
AB_ROUNDS=3 bash bench/ab_env.sh "mark:" "elemt:PMD_FORK_ELEMT=1" > gpurun_out/ab_elemt.txt 2>&1 &&
AB_ROUNDS=2 AB_ARGS="--dtype fp8" bash bench/ab_env.sh "mark:" "elemt:PMD_FORK_ELEMT=1" > gpurun_out/ab_elemt_fp8.txt 2>&1
