# round-5 GPU step 17: LDS-heavy weight-gradient variants vs main-stream co-residency (A/B)
set -o pipefail
mkdir -p gpurun_out
export PMD_NO_AUTOBUILD=1
AB_ROUNDS=2 bash bench/ab_env.sh "base:" "m4:PMD_WGRAD_MAP4=1" "m45:PMD_WGRAD_MAP4=1,PMD_WGRAD_MAP5=1" "m456:PMD_WGRAD_MAP4=1,PMD_WGRAD_MAP5=1,PMD_WGRAD_MAP6=1" "m46:PMD_WGRAD_MAP4=1,PMD_WGRAD_MAP6=1" > gpurun_out/ab_map.txt 2>&1
