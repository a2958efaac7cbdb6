# round-5 GPU step 15: bnlin coefficient kernel with K slices (tests + kernel trace) and the dgrad
# epilogue operand prefetch variants (PMD_EPI_PF=1/2) A/B
set -o pipefail
mkdir -p gpurun_out
export PMD_NO_AUTOBUILD=1
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_bnlin_gpu.py > gpurun_out/t15.log 2>&1 &&
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" &&
timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/kt15 -o run -- python3 bench.py --steps 16 --warmup 6 > gpurun_out/kt15.log 2>&1 &&
bash bench/ab_so.sh base pf1 pf2 > gpurun_out/ab_pf.txt 2>&1
