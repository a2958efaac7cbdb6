# round-5 GPU step 26: weight images refreshed on the side stream next to the stem (A/B)
set -o pipefail
mkdir -p gpurun_out
export PMD_NO_AUTOBUILD=1
AB_ROUNDS=3 bash bench/ab_env.sh "base:" "wside:PMD_WPREP_SIDE=1" > gpurun_out/ab_wside.txt 2>&1
