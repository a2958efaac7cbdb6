# round-5 GPU step 34: dgrad weight images on the side stream during the forward (PMD_SPLIT_WPREP) A/B
set -o pipefail
mkdir -p gpurun_out
export PMD_NO_AUTOBUILD=1
AB_ROUNDS=3 bash bench/ab_env.sh "base:" "split:PMD_SPLIT_WPREP=1" > gpurun_out/ab_split.txt 2>&1
