set -o pipefail
mkdir -p gpurun_out
export PMD_NO_AUTOBUILD=1
timeout -k 10 300 python -m pytest tests/test_fp8_gpu.py -x -q > gpurun_out/fp8_tests.log 2>&1
