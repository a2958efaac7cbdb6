export PMD_NO_AUTOBUILD=1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
bash bench/gpu_run.sh \
 "xgmitests:400:python -u -m pytest tests/test_xgmi_gpu.py tests/test_multirank_gpu.py -x -q --timeout 200 --timeout-method thread" \
 "r50:200:python bench.py --steps 30 --warmup 10" \
 "reh:200:python bench.py --steps 30 --warmup 10 --dp_rehearsal" \
 "reh_c10d:200:python bench.py --steps 30 --warmup 10 --dp_rehearsal --comm c10d" \
 "r50b:200:python bench.py --steps 30 --warmup 10" \
 "reh2:200:python bench.py --steps 30 --warmup 10 --dp_rehearsal" \
 "r152:300:python bench.py --steps 20 --warmup 8 --model resnet152" \
 "r152_reh:300:python bench.py --steps 20 --warmup 8 --model resnet152 --dp_rehearsal" \
 "w2:400:python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --same_device --backend gloo --syncbn_comm xgmi --steps 6 --warmup 3 --batch 64" \
 "prof_reh:300:rocprofv3 --kernel-trace --stats -d gpurun_out/prof_reh6 -o run -- python3 bench.py --steps 10 --warmup 5 --dp_rehearsal"
