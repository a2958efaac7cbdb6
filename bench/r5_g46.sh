# round-5 GPU step 46: side-stream join lag 0 (join at the end of the same block) vs 1 (default)
set -o pipefail
mkdir -p gpurun_out
export PMD_NO_AUTOBUILD=1
AB_ROUNDS=3 bash bench/ab_env.sh "d1:" "d0:PMD_WGRAD_DEFER=0" > gpurun_out/ab_defer0.txt 2>&1
