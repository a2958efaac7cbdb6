# round-5 GPU step 27: final-tree PMC passes + two-stream kernel trace with stats (bytes budget / rocprof stats)
set -o pipefail
mkdir -p gpurun_out
export PMD_NO_AUTOBUILD=1
bash bench/pmc_step.sh gpurun_out/pmc27 &&
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" &&
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/ks27 -o run -- python3 bench.py --steps 10 --warmup 5 > gpurun_out/ks27.log 2>&1
