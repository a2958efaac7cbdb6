# round-5 GPU step 43: fork/join as stream memory operations (write/wait value, ring mode 3): microbench,
# exactness, then the step A/B against the fence-less event ring (mode 1, the default)
set -o pipefail
mkdir -p gpurun_out
export PMD_NO_AUTOBUILD=1
timeout -k 10 120 python bench/event_fence.py > gpurun_out/event_fence3.txt 2>&1 &&
AB_ROUNDS=3 bash bench/ab_env.sh "m1:" "m3:PMD_FORK_EVENTS=3" > gpurun_out/ab_ring3.txt 2>&1
