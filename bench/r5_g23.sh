# round-5 GPU step 23: tuned conv choices remapped in the full step (co-residency with the side stream)
set -o pipefail
mkdir -p gpurun_out
export PMD_NO_AUTOBUILD=1
AB_ROUNDS=2 bash bench/ab_env.sh "base:" "d2to3:PMD_CONV_REMAP=d2:3" "d2to4:PMD_CONV_REMAP=d2:4" "d4to0:PMD_CONV_REMAP=d4:0" "d4to1:PMD_CONV_REMAP=d4:1" "f2to3:PMD_CONV_REMAP=f2:3" > gpurun_out/ab_remap.txt 2>&1
