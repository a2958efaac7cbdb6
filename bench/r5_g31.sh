# round-5 GPU step 31: shift instead of division in the general conv loader (stem): tests + trace + bench
set -o pipefail
mkdir -p gpurun_out
export PMD_NO_AUTOBUILD=1
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_stem_s2d_gpu.py tests/test_kernels_gpu.py -k "stem or conv_fwd_dgrad or pipeline or oracle or big_tiles" > gpurun_out/t31.log 2>&1 &&
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" &&
timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/kt31 -o run -- python3 bench.py --steps 16 --warmup 6 > gpurun_out/kt31.log 2>&1 &&
cd "$GRAFT_REPO_ROOT" && AB_ROUNDS=2 bash bench/ab_env.sh "new:" > gpurun_out/ab31.txt 2>&1
