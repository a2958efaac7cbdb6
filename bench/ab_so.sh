# A/B the full training step across prebuilt extension variants ($AB_DIR/so_<name>.so,
# AB_DIR defaults to abso), interleaved rounds in one box session: bash bench/ab_so.sh name1 name2 ...
# (AB_ARGS: extra bench.py arguments, e.g. "--dtype fp8")
set -o pipefail
mkdir -p gpurun_out
export PMD_NO_AUTOBUILD=1
export PMD_ALLOW_VARIANT=1   # the variants are the point here (ops/native.py refuses them otherwise)
SO=pytorch_multiprocessing_distributed_amd/_C.cpython-310-x86_64-linux-gnu.so
D=${AB_DIR:-abso}
cp $SO $D/so_current_backup.so
for round in 1 2; do
  for v in "$@"; do
    cp $D/so_$v.so $SO
    r=$(timeout -k 10 200 python bench.py --steps 30 --warmup 10 ${AB_ARGS:-} 2>/dev/null | tail -1) || exit 1
    echo "$round $v $(echo "$r" | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
  done
done
cp $D/so_current_backup.so $SO
