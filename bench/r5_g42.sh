# round-5 GPU step 42: full GPU suite with the fork/join ring as the default; step A/B ring vs torch events
set -o pipefail
mkdir -p gpurun_out
export PMD_NO_AUTOBUILD=1
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_stream_events_gpu.py > gpurun_out/sev_tests.txt 2>&1 &&
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_full.txt 2>&1 &&
AB_ROUNDS=3 bash bench/ab_env.sh "torch:PMD_FORK_EVENTS=-1" "ring:" > gpurun_out/ab_ring.txt 2>&1
