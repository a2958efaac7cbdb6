export PMD_NO_AUTOBUILD=1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/tables
bash bench/gpu_run.sh \
 "r50:200:python bench.py --steps 30 --warmup 10" \
 "reh:200:python bench.py --steps 30 --warmup 10 --dp_rehearsal" \
 "reh_c10d:200:python bench.py --steps 30 --warmup 10 --dp_rehearsal --comm c10d" \
 "r152:300:python bench.py --steps 20 --warmup 8 --model resnet152" \
 "r152_reh:300:python bench.py --steps 20 --warmup 8 --model resnet152 --dp_rehearsal" \
 "r152_reh_c10d:300:python bench.py --steps 20 --warmup 8 --model resnet152 --dp_rehearsal --comm c10d" \
 "tune_cifar:600:python bench/make_tune_table.py --runs 5 --out pytorch_multiprocessing_distributed_amd/ops/tables/res_cifar_bs32_gfx950.json -- --model res --batch 32 --image 32 --classes 10 --stem cifar" \
 "cp_table:30:cp pytorch_multiprocessing_distributed_amd/ops/tables/res_cifar_bs32_gfx950.json gpurun_out/tables/" \
 "cifar:200:python bench.py --steps 50 --warmup 10 --model res --batch 32 --image 32 --classes 10 --stem cifar"
(while sleep 20; do date >> gpurun_out/hb_w2.txt; done) &
HB=$!
bash bench/gpu_run.sh \
 "prof_w2:240:rocprofv3 --kernel-trace -d gpurun_out/prof_w2q2 -o run -- python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29534 bench.py --gpus 2 --same_device --backend gloo --syncbn_comm xgmi --steps 3 --warmup 2 --batch 32"
rc=$?
kill $HB
exit $rc
