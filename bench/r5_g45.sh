# round-5 GPU step 45: side-stream join lag (PMD_WGRAD_DEFER: 1 default, 3, 99 = only at the end of backward) A/B, bf16 and rehearsal
set -o pipefail
mkdir -p gpurun_out
export PMD_NO_AUTOBUILD=1
AB_ROUNDS=2 bash bench/ab_env.sh "d1:" "d3:PMD_WGRAD_DEFER=3" "d99:PMD_WGRAD_DEFER=99" > gpurun_out/ab_defer.txt 2>&1 &&
AB_ROUNDS=1 AB_ARGS="--dp_rehearsal" bash bench/ab_env.sh "d1:" "d3:PMD_WGRAD_DEFER=3" "d99:PMD_WGRAD_DEFER=99" > gpurun_out/ab_defer_reh.txt 2>&1
