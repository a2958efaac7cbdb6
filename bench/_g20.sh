export PMD_NO_AUTOBUILD=1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
bash bench/gpu_run.sh \
 "on0:300:python bench.py --steps 30 --warmup 10 --tune_table online" \
 "on1:300:PMD_TUNE_MF32=1 PMD_CONV_AUTOTUNE_LOG=1 python bench.py --steps 30 --warmup 10 --tune_table online" \
 "on0b:300:python bench.py --steps 30 --warmup 10 --tune_table online" \
 "on1b:300:PMD_TUNE_MF32=1 python bench.py --steps 30 --warmup 10 --tune_table online" \
 "tab:200:python bench.py --steps 30 --warmup 10"
