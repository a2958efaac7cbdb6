export PMD_NO_AUTOBUILD=1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
bash bench/gpu_run.sh \
 "reh:200:python bench.py --steps 30 --warmup 10 --dp_rehearsal" \
 "reh_noov:200:PMD_SYNCBN_OVERLAP=0 python bench.py --steps 30 --warmup 10 --dp_rehearsal" \
 "r50:200:python bench.py --steps 30 --warmup 10" \
 "reh_noov2:200:PMD_SYNCBN_OVERLAP=0 python bench.py --steps 30 --warmup 10 --dp_rehearsal" \
 "reh2:200:python bench.py --steps 30 --warmup 10 --dp_rehearsal" \
 "r152_noov:300:PMD_SYNCBN_OVERLAP=0 python bench.py --steps 20 --warmup 8 --model resnet152 --dp_rehearsal" \
 "w2_noov:400:PMD_SYNCBN_OVERLAP=0 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --same_device --backend gloo --syncbn_comm xgmi --steps 6 --warmup 3 --batch 64" \
 "prof_noov:300:PMD_SYNCBN_OVERLAP=0 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_reh_noov -o run -- python3 bench.py --steps 10 --warmup 5 --dp_rehearsal"
