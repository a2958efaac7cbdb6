# round-5 GPU step 48: stream priorities on the final tree (side stream at normal priority; all step streams normal)
set -o pipefail
mkdir -p gpurun_out
export PMD_NO_AUTOBUILD=1
AB_ROUNDS=2 bash bench/ab_env.sh "base:" "wprio0:PMD_WGRAD_PRIO=0" "sprio0:PMD_STREAM_PRIO=0" > gpurun_out/ab_prio.txt 2>&1
