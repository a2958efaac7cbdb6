# round-5 GPU step 39: weight-prep tile walk with all 16 rows' loads in flight -- separate passes
# (tile9) vs one mode-3 walk (fused3) vs the 4-in-flight separate passes (tile8): step A/B + kernel traces
set -o pipefail
mkdir -p gpurun_out
export PMD_NO_AUTOBUILD=1 PMD_ALLOW_VARIANT=1
SO=pytorch_multiprocessing_distributed_amd/_C.cpython-310-x86_64-linux-gnu.so
bash bench/ab_so.sh tile8 tile9 fused3 > gpurun_out/ab_w39.txt 2>&1 &&
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" &&
for v in tile9 fused3; do
  cp abso/so_$v.so $SO &&
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/wt_$v -o run -- python3 bench.py --steps 12 --warmup 6 > gpurun_out/wt_$v.log 2>&1 || exit 1
done
