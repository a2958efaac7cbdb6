set -o pipefail
R=$(pwd)
mkdir -p gpurun_out
export PMD_NO_AUTOBUILD=1
cd /tmp && export TMPDIR=/tmp && \
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof9 -o run -- python $R/bench.py --steps 5 --warmup 3 > $R/gpurun_out/prof9.log 2>&1
