# A/B: autotuned at step 0 vs a loaded tuning table, interleaved rounds
set -o pipefail
export PMD_NO_AUTOBUILD=1
T=pytorch_multiprocessing_distributed_amd/tuning/r50_bs256_mi355x.json
for round in 1 2 3; do
  r=$(timeout -k 10 200 python bench.py --steps 30 --warmup 10 2>/dev/null | tail -1) || exit 1
  echo "$round auto $(echo "$r" | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
  r=$(timeout -k 10 200 python bench.py --steps 30 --warmup 10 --tune_table $T 2>/dev/null | tail -1) || exit 1
  echo "$round table $(echo "$r" | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
done
