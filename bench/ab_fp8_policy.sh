# fp8 conv policy A/B on the full step: bf16, fp8 on every conv with Kg >= 128
# (PMD_FP8_CONVS=all), fp8 on the 3x3 convs only (default), interleaved rounds
set -o pipefail
export PMD_NO_AUTOBUILD=1
for r in 1 2; do
  for cfg in "bf16 x" "fp8 all" "fp8 spatial"; do
    set -- $cfg
    v=$(PMD_FP8_CONVS=$2 timeout -k 10 200 python bench.py --steps 30 --warmup 10 --dtype $1 2>/dev/null | tail -1) || exit 1
    echo "$r $1 $2 $(echo "$v" | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
  done
done
