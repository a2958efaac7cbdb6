# round-5 GPU step 29: the 32x32x16-MFMA tile (candidate 13) in place of tuned choices (A/B)
set -o pipefail
mkdir -p gpurun_out
export PMD_NO_AUTOBUILD=1
AB_ROUNDS=2 bash bench/ab_env.sh "base:" "f5mf:PMD_CONV_REMAP=f5:13" "f2mf:PMD_CONV_REMAP=f2:13" "d1mf:PMD_CONV_REMAP=d1:13" "d2mf:PMD_CONV_REMAP=d2:13" "f1mf:PMD_CONV_REMAP=f1:13" > gpurun_out/ab_mf32.txt 2>&1
