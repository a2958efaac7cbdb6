# steady-state kernel trace of the fp8 (config 5) step
set -o pipefail
mkdir -p gpurun_out
export PMD_NO_AUTOBUILD=1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && rm -rf gpurun_out/prof8 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof8 -o run -- python3 bench.py --dtype fp8 --steps 6 --warmup 4 > gpurun_out/prof8.log 2>&1
