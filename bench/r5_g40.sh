# round-5 GPU step 40: cost of a cross-stream fork by event kind (microbench + hand-off exactness),
# then the full step with the weight-gradient fork/join points on the native event ring, per fence mode
set -o pipefail
mkdir -p gpurun_out
export PMD_NO_AUTOBUILD=1
timeout -k 10 300 python bench/event_fence.py > gpurun_out/event_fence.txt 2>&1 &&
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_stream_events_gpu.py > gpurun_out/sev_tests.txt 2>&1 &&
AB_ROUNDS=2 bash bench/ab_env.sh "torch:" "m0:PMD_FORK_EVENTS=0" "m1:PMD_FORK_EVENTS=1" "m2:PMD_FORK_EVENTS=2" > gpurun_out/ab_forkev.txt 2>&1
