set -o pipefail
mkdir -p gpurun_out
export PMD_NO_AUTOBUILD=1
step() { local name=$1 secs=$2; shift 2; echo "[call4] $(date +%T) $name"; timeout -k 10 $secs "$@" > gpurun_out/c4_$name.log 2>&1; local rc=$?; tail -4 gpurun_out/c4_$name.log; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "[call4] $name rc=$rc: stopping"; exit $rc; fi; return 0; }
step tests 420 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_model_oracle_gpu.py tests/test_multirank_gpu.py
step w2 240 python3 bench.py --gpus 2 --backend gloo --same_device --timeline --steps 5 --warmup 3
step w4 300 python3 bench.py --gpus 4 --backend gloo --same_device --steps 3 --warmup 2
GPU_MAX_HW_QUEUES=1 step w4q1 300 python3 bench.py --gpus 4 --backend gloo --same_device --steps 3 --warmup 2
step pmcwino 400 bash bench/pmc_step.sh gpurun_out/pmc_wino -- python3 bench/winograd_bench.py --batch 256
for cfg in "64 56 64 3 1:1" "64 56 64 3 1:0" "64 56 256 1 1:1" "1024 14 256 1 1:1" "1024 14 256 1 1:4" "256 14 256 3 1:4"; do
  shp=${cfg%%:*}; wi=${cfg#*:}; tag=$(echo "$shp" | tr ' ' '_')_w$wi
  PMD_WGRAD_AUTOTUNE=0 step pmcw_$tag 200 bash bench/pmc_step.sh gpurun_out/pmc_wg/$tag -- python3 bench/conv_one.py $shp --pass wgrad --wimpl $wi --iters 8
done
echo "[call4] done"
