# Kernel trace of 6 bench steps (rocpd DB comes back for per-dispatch analysis).
set -o pipefail
mkdir -p gpurun_out
export PMD_NO_AUTOBUILD=1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run -- python3 bench.py --steps 6 --warmup 4 > gpurun_out/prof.log 2>&1
