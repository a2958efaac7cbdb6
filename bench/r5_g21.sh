# round-5 GPU step 21: kernel + HIP API trace of the bf16 step (host enqueue lag vs GPU gaps on the main stream)
set -o pipefail
mkdir -p gpurun_out
export PMD_NO_AUTOBUILD=1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 240 rocprofv3 --kernel-trace --hip-trace --output-format csv -d gpurun_out/kt21 -o run -- python3 bench.py --steps 12 --warmup 6 > gpurun_out/kt21.log 2>&1
