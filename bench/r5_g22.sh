# round-5 GPU step 22: kernel trace of the W=1 DP rehearsal (vs the plain step's trace)
set -o pipefail
mkdir -p gpurun_out
export PMD_NO_AUTOBUILD=1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/kt22r -o run -- python3 bench.py --steps 16 --warmup 6 --dp_rehearsal > gpurun_out/kt22r.log 2>&1 &&
timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/kt22p -o run -- python3 bench.py --steps 16 --warmup 6 > gpurun_out/kt22p.log 2>&1
