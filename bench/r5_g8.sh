set -o pipefail
mkdir -p gpurun_out
export PMD_NO_AUTOBUILD=1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/klin -o run -- python3 bench.py --steps 10 --warmup 5 > gpurun_out/klin.log 2>&1 &&
PMD_BNLIN=0 timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/kelt -o run -- python3 bench.py --steps 10 --warmup 5 > gpurun_out/kelt.log 2>&1
