# GPU tests on the new build, then interleaved A/B of the full step vs the previous build.
set -o pipefail
mkdir -p gpurun_out
export PMD_NO_AUTOBUILD=1
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 && \
bash bench/ab_so.sh "$@" > gpurun_out/ab.log 2>&1
