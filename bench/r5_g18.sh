# round-5 GPU step 18: kernel traces, two-stream vs single-stream step (contention attribution)
set -o pipefail
mkdir -p gpurun_out
export PMD_NO_AUTOBUILD=1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/kt18a -o run -- python3 bench.py --steps 16 --warmup 6 > gpurun_out/kt18a.log 2>&1 &&
PMD_WGRAD_STREAM=0 timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/kt18b -o run -- python3 bench.py --steps 16 --warmup 6 > gpurun_out/kt18b.log 2>&1
