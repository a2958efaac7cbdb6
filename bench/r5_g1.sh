set -o pipefail
mkdir -p gpurun_out
export PMD_NO_AUTOBUILD=1
timeout -k 10 600 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_xgmi_gpu.py tests/test_distributed_gpu.py > gpurun_out/t1.log 2>&1 &&
timeout -k 10 240 python bench.py --steps 20 --warmup 5 > gpurun_out/b1.jsonl 2> gpurun_out/b1.err &&
timeout -k 10 240 python bench.py --steps 20 --warmup 5 --dp_rehearsal >> gpurun_out/b1.jsonl 2>> gpurun_out/b1.err
