export PMD_NO_AUTOBUILD=1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
bash bench/gpu_run.sh \
 "r50:200:python bench.py --steps 30 --warmup 10" \
 "reh:200:python bench.py --steps 30 --warmup 10 --dp_rehearsal" \
 "reh2:200:python bench.py --steps 30 --warmup 10 --dp_rehearsal" \
 "reh_c10d:200:python bench.py --steps 30 --warmup 10 --dp_rehearsal --comm c10d" \
 "reh3:200:python bench.py --steps 30 --warmup 10 --dp_rehearsal" \
 "mr:400:python -u -m pytest tests/test_multirank_gpu.py tests/test_xgmi_gpu.py tests/test_distributed_gpu.py -x -q --timeout 200 --timeout-method thread" \
 "prof_reh:300:rocprofv3 --kernel-trace -d gpurun_out/prof_reh8 -o run -- python3 bench.py --steps 10 --warmup 5 --dp_rehearsal" || exit $?
(while sleep 20; do date >> gpurun_out/hb_w2.txt; done) &
HB=$!
bash bench/gpu_run.sh \
 "prof_w2:240:rocprofv3 --kernel-trace -d gpurun_out/prof_w2q5 -o run_%pid% -- python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29534 bench.py --gpus 2 --same_device --backend gloo --syncbn_comm xgmi --steps 3 --warmup 2 --batch 32"
rc=$?
kill $HB
exit $rc
