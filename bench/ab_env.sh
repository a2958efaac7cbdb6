# A/B the full training step across environment settings, interleaved rounds in one box
# session:  bash bench/ab_env.sh "base:" "r1_256:PMD_WGRAD_BLOCKS_R1=256" "x:A=1,B=2" ...
# (name:comma-separated VAR=value list; an empty list = the defaults)
set -o pipefail
mkdir -p gpurun_out
export PMD_NO_AUTOBUILD=1
ROUNDS=${AB_ROUNDS:-2}
for round in $(seq 1 $ROUNDS); do
  for spec in "$@"; do
    name=${spec%%:*}; envs=${spec#*:}
    r=$(env ${envs//,/ }  timeout -k 10 200 python bench.py --steps 30 --warmup 10 ${AB_ARGS:-} 2>/dev/null | tail -1) || exit 1
    echo "$round $name $(echo "$r" | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
  done
done
