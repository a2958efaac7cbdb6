export PMD_NO_AUTOBUILD=1
bash bench/gpu_run.sh \
 "tune_cifar:900:python bench/make_tune_table.py --runs 5 --out pytorch_multiprocessing_distributed_amd/ops/tables/res_cifar_bs32_gfx950.json -- --model res --batch 32 --image 32 --classes 10 --stem cifar"
mkdir -p gpurun_out/tables && cp pytorch_multiprocessing_distributed_amd/ops/tables/res_cifar_bs32_gfx950.json gpurun_out/tables/ 2>/dev/null; true
