set -o pipefail
mkdir -p gpurun_out
export PMD_NO_AUTOBUILD=1
timeout -k 10 300 python -m pytest tests/test_xgmi_gpu.py tests/test_distributed_gpu.py -x -q -s > gpurun_out/xgmi_test.log 2>&1
