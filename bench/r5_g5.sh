set -o pipefail
bash bench/pmc_lds.sh base episw2 swz1 > gpurun_out/pmc_lds.log 2>&1 &&
AB_DIR=abso bash bench/ab_so.sh base episw2 swz1 > gpurun_out/ab_lds.txt 2>&1
