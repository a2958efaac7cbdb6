# round-5 GPU step 28: re-vote the ResNet-50 bs256 tuning table on the current kernels, then A/B it in the step
set -o pipefail
mkdir -p gpurun_out
export PMD_NO_AUTOBUILD=1
timeout -k 10 700 python bench/make_tune_table.py --runs 5 --out gpurun_out/r50_revote.json > gpurun_out/revote.log 2>&1 &&
AB_ROUNDS=3 bash bench/ab_env.sh "old:" > gpurun_out/ab_tt_old.txt 2>&1 &&
AB_ROUNDS=3 AB_ARGS="--tune_table gpurun_out/r50_revote.json" bash bench/ab_env.sh "new:" > gpurun_out/ab_tt_new.txt 2>&1
