set -o pipefail
mkdir -p gpurun_out
export PMD_NO_AUTOBUILD=1
timeout -k 10 120 python bench/pool_bench.py > gpurun_out/pool_new.log 2>&1 && \
cp build/oldso/_C_old.so pytorch_multiprocessing_distributed_amd/_C.cpython-310-x86_64-linux-gnu.so && \
timeout -k 10 120 python bench/pool_bench.py > gpurun_out/pool_old.log 2>&1
