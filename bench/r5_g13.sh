# round-5 GPU step 13: side-stream occupancy caps (PMD_WGRAD_LDS_PAD, PMD_WGRAD_HALO_BLOCKS) A/B
set -o pipefail
mkdir -p gpurun_out
export PMD_NO_AUTOBUILD=1
AB_ROUNDS=3 bash bench/ab_env.sh "base:" "pad20k:PMD_WGRAD_LDS_PAD=20000" "pad34k:PMD_WGRAD_LDS_PAD=34000" "halo128:PMD_WGRAD_HALO_BLOCKS=128" > gpurun_out/ab_ldspad.txt 2>&1
