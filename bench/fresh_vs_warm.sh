#!/bin/bash
# Fresh-lease reproduction of the driver's bench command (run as the FIRST GPU
# process of a gpurun call), then the same command warm, then with the committed
# tuning table, then a longer window, then a rocprofv3 kernel-stats pass of the
# exact driver command.  Each step has its own limit; stops at the first crash.
#   gpurun -- bash bench/fresh_vs_warm.sh <tag> [extra bench args]
set -u
tag=${1:-fw}; shift || true
extra="$*"
mkdir -p gpurun_out
export TMPDIR=/tmp
run() {  # name, seconds, command...
  local name=$1 secs=$2; shift 2
  echo "[fw] $(date +%T) $name: $*"
  timeout -k 10 "$secs" "$@" > "gpurun_out/${tag}_$name.out" 2> "gpurun_out/${tag}_$name.err"
  local rc=$?
  tail -c 600 "gpurun_out/${tag}_$name.out"; echo
  if [ $rc -ne 0 ]; then echo "[fw] $name rc=$rc"; tail -20 "gpurun_out/${tag}_$name.err"; exit $rc; fi
}
PMD_CONV_AUTOTUNE_LOG=1 run fresh1 240 python3 bench.py --gpus 1 --steps 20 --warmup 5 $extra
PMD_CONV_AUTOTUNE_LOG=1 run warm2 240 python3 bench.py --gpus 1 --steps 20 --warmup 5 $extra
run warm3 240 python3 bench.py --gpus 1 --steps 20 --warmup 5 $extra
run online4 240 python3 bench.py --gpus 1 --steps 20 --warmup 5 --tune_table online $extra
run long100 240 python3 bench.py --gpus 1 --steps 100 --warmup 20 $extra
cd /tmp && cd - > /dev/null
run prof 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${tag}_prof -o run -- python3 bench.py --gpus 1 --steps 20 --warmup 5 $extra
echo "[fw] done"
