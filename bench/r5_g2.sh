# round-5 GPU step 2: copy attribution, PMC step counters, two-stream kernel trace
set -o pipefail
mkdir -p gpurun_out
export PMD_NO_AUTOBUILD=1
timeout -k 10 200 python bench/copy_sites.py > gpurun_out/copy_sites.txt 2> gpurun_out/copy_sites.err &&
bash bench/pmc_step.sh gpurun_out/pmc5 &&
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" &&
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/ks5 -o run -- python3 bench.py --steps 10 --warmup 5 > gpurun_out/ks5.log 2>&1
