# round-5 GPU step 47: projection-shortcut weight gradient on the final conv's fork (PMD_SC_EARLY) -- oracles, step A/B
set -o pipefail
mkdir -p gpurun_out
export PMD_NO_AUTOBUILD=1
PMD_SC_EARLY=1 timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_model_oracle_gpu.py tests/test_fp8_gpu.py tests/test_distributed_gpu.py tests/test_stream_events_gpu.py > gpurun_out/sc_tests.txt 2>&1 &&
AB_ROUNDS=3 bash bench/ab_env.sh "base:" "sc:PMD_SC_EARLY=1" > gpurun_out/ab_sc.txt 2>&1 &&
AB_ROUNDS=1 AB_ARGS="--dtype fp8" bash bench/ab_env.sh "base:" "sc:PMD_SC_EARLY=1" > gpurun_out/ab_sc_fp8.txt 2>&1 &&
AB_ROUNDS=1 AB_ARGS="--dp_rehearsal" bash bench/ab_env.sh "base:" "sc:PMD_SC_EARLY=1" > gpurun_out/ab_sc_reh.txt 2>&1
