export PMD_NO_AUTOBUILD=1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
bash bench/gpu_run.sh \
 "a1:200:python bench.py --steps 30 --warmup 10" \
 "b1:200:PMD_WGRAD_PRIO=0 python bench.py --steps 30 --warmup 10" \
 "c1:200:PMD_STREAM_PRIO=0 python bench.py --steps 30 --warmup 10" \
 "a2:200:python bench.py --steps 30 --warmup 10" \
 "b2:200:PMD_WGRAD_PRIO=0 python bench.py --steps 30 --warmup 10" \
 "c2:200:PMD_STREAM_PRIO=0 python bench.py --steps 30 --warmup 10" \
 "rb1:200:PMD_WGRAD_PRIO=0 python bench.py --steps 30 --warmup 10 --dp_rehearsal" \
 "f8:200:python bench.py --steps 30 --warmup 10 --dtype fp8" \
 "r152:300:python bench.py --steps 20 --warmup 8 --model resnet152"
