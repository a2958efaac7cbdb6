# A/B the full training step across environment-variable variants, interleaved
# rounds in one box session:  bash bench/ab_env.sh "name:VAR=v VAR2=w" "base:" ...
set -o pipefail
mkdir -p gpurun_out
export PMD_NO_AUTOBUILD=1
for round in 1 2; do
  for spec in "$@"; do
    name="${spec%%:*}"; envs="${spec#*:}"
    r=$(env $envs timeout -k 10 200 python bench.py --steps 30 --warmup 10 2>/dev/null | tail -1) || exit 1
    echo "$round $name $(echo "$r" | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
  done
done
