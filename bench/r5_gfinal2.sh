# round-5 final records on the final tree: bench rows (driver command first) + kernel-trace stats
set -o pipefail
mkdir -p gpurun_out
export PMD_NO_AUTOBUILD=1
bash bench/r5_gfinal_bench.sh &&
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" &&
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/final2_prof -o run -- python3 bench.py --steps 10 --warmup 5 > gpurun_out/final2_prof.log 2>&1
