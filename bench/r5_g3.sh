# round-5 GPU step 3: kernel traces of (a) the HIP-graph replay of the step, (b) the W=1 DP rehearsal
set -o pipefail
mkdir -p gpurun_out
export PMD_NO_AUTOBUILD=1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/kgraph -o run -- python3 bench.py --steps 10 --warmup 5 --graph > gpurun_out/kgraph.log 2>&1 &&
timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/kreh -o run -- python3 bench.py --steps 10 --warmup 5 --dp_rehearsal > gpurun_out/kreh.log 2>&1
