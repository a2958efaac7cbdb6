# round-5 GPU step 4: tuning-table coverage, voted BasicBlock/ImageNet table, stock comparator
set -o pipefail
mkdir -p gpurun_out
export PMD_NO_AUTOBUILD=1
timeout -k 10 300 python bench/tune_coverage.py resnet34 resnet18full resnet101 resnet152 > gpurun_out/cov_before.txt 2>&1 &&
timeout -k 10 900 python bench/make_tune_table.py --runs 5 --out gpurun_out/basic_in224_bs256_gfx950.json -- --model resnet34 > gpurun_out/tune_r34.log 2>&1 &&
cp gpurun_out/basic_in224_bs256_gfx950.json pytorch_multiprocessing_distributed_amd/ops/tables/ &&
timeout -k 10 300 python bench/tune_coverage.py resnet34 resnet18full resnet50 > gpurun_out/cov_after.txt 2>&1 &&
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --with_stock > gpurun_out/stock.jsonl 2> gpurun_out/stock.err
