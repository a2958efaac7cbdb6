# stem pool-backward reduce rows-per-block A/B: kernel trace of each variant (stem kernels only matter)
set -o pipefail
mkdir -p gpurun_out
export PMD_NO_AUTOBUILD=1
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q -k "stem" --timeout 120 --timeout-method thread > gpurun_out/stem_tests.log 2>&1 && \
bash bench/ab_so.sh rpb2 rpb4 rpb8 rpb16 > gpurun_out/ab_rpb.log 2>&1
