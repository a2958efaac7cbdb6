# round-5 GPU step 20: fp8 vs bf16 in one lease + fp8 kernel trace
set -o pipefail
mkdir -p gpurun_out
export PMD_NO_AUTOBUILD=1
AB_ROUNDS=2 bash bench/ab_env.sh "bf16:" > gpurun_out/ab_dt_bf16.txt 2>&1 &&
AB_ROUNDS=2 AB_ARGS="--dtype fp8" bash bench/ab_env.sh "fp8:" > gpurun_out/ab_dt_fp8.txt 2>&1 &&
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" &&
timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/kt20 -o run -- python3 bench.py --steps 16 --warmup 6 --dtype fp8 > gpurun_out/kt20.log 2>&1
