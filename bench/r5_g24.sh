# round-5 GPU step 24: halo-image 3x3 kernel for the stride-1 3x3 convs in the full step (A/B)
set -o pipefail
mkdir -p gpurun_out
export PMD_NO_AUTOBUILD=1
AB_ROUNDS=2 bash bench/ab_env.sh "base:" "hf11:PMD_CONV_HALO=f:11" "hf12:PMD_CONV_HALO=f:12" "hd11:PMD_CONV_HALO=d:11" "hd12:PMD_CONV_HALO=d:12" > gpurun_out/ab_halo.txt 2>&1
