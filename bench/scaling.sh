#!/usr/bin/env bash
# Weak-scaling sweep of the flagship benchmark on one node: N = 1, 2, 4, 8 GPUs
# (per-GPU batch 256, ResNet-50 224x224 bf16, SyncBN + bucketed RCCL all-reduce).
# Prints one JSON line per N and a summary with scaling efficiency ips(N)/(N*ips(1)).
#   bash bench/scaling.sh [STEPS] [WARMUP]
set -euo pipefail
STEPS=${1:-30}
WARMUP=${2:-10}
cd "$(dirname "$0")/.."
out=$(mktemp)
for N in 1 2 4 8; do
  if [ "$N" -gt "$(python -c 'import torch; print(torch.cuda.device_count())')" ]; then break; fi
  if [ "$N" -eq 1 ]; then
    timeout -k 10 900 python bench.py --gpus 1 --steps "$STEPS" --warmup "$WARMUP" | tail -n 1 | tee -a "$out"
  else
    timeout -k 10 900 python -m torch.distributed.run --nnodes=1 --nproc-per-node "$N" \
      --master-addr 127.0.0.1 --master-port $((29600 + N)) bench.py --gpus "$N" \
      --steps "$STEPS" --warmup "$WARMUP" | tail -n 1 | tee -a "$out"
  fi
done
python - "$out" <<'PY'
import json, sys
rows = [json.loads(l) for l in open(sys.argv[1]) if l.startswith("{")]
base = next((r["value"] for r in rows if r["n_gpus"] == 1), None)
for r in rows:
    eff = r["value"] / (r["n_gpus"] * base) if base else float("nan")
    print(f"N={r['n_gpus']}: {r['value']:.1f} img/s  ({r['ms_per_step']:.2f} ms/step)  scaling eff {eff:.3f}")
PY
