export PMD_NO_AUTOBUILD=1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
bash bench/gpu_run.sh \
 "cifar:200:python bench.py --steps 100 --warmup 20 --model res --batch 32 --image 32 --classes 10 --stem cifar" \
 "cifar_graph:200:python bench.py --steps 100 --warmup 20 --model res --batch 32 --image 32 --classes 10 --stem cifar --graph" \
 "r50_graph:200:python bench.py --steps 30 --warmup 10 --graph" \
 "pmc_bf16:500:bash bench/pmc_step.sh gpurun_out/pmc_r04" || exit $?
(while sleep 20; do date >> gpurun_out/hb_w2.txt; done) &
HB=$!
bash bench/gpu_run.sh \
 "prof_w2:240:rocprofv3 --kernel-trace -d gpurun_out/prof_w2q3 -o run_%pid% -- python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29534 bench.py --gpus 2 --same_device --backend gloo --syncbn_comm xgmi --steps 3 --warmup 2 --batch 32"
rc=$?
kill $HB
exit $rc
