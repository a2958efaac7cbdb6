# round-5 GPU step 41: fork/join on the native ring by default -- oracle tests; step A/B of
# fork batching (PMD_FORK_BATCH) and torch events
set -o pipefail
mkdir -p gpurun_out
export PMD_NO_AUTOBUILD=1
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_stream_events_gpu.py \
  tests/test_bnlin_gpu.py tests/test_model_oracle_gpu.py tests/test_distributed_gpu.py > gpurun_out/fork_tests.txt 2>&1 &&
AB_ROUNDS=2 bash bench/ab_env.sh "torch:PMD_FORK_EVENTS=-1" "b1:" "b2:PMD_FORK_BATCH=2" "b3:PMD_FORK_BATCH=3" > gpurun_out/ab_forkbatch.txt 2>&1
