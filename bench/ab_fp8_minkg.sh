set -o pipefail
export PMD_NO_AUTOBUILD=1
for r in 1 2; do
  for kg in 0 128; do
    v=$(PMD_FP8_MIN_KG=$kg timeout -k 10 200 python bench.py --steps 30 --warmup 10 --dtype fp8 2>/dev/null | tail -1) || exit 1
    echo "$r minkg=$kg $(echo "$v" | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
  done
done
