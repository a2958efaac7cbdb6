set -o pipefail
mkdir -p gpurun_out
rocm-smi > gpurun_out/smi.txt 2>&1 || true
rocminfo | grep -E "Name:|Compute Unit|gfx" | head -20 > gpurun_out/rocminfo.txt 2>&1 || true
timeout -k 10 500 python bench/comparator_torch.py --steps 20 --warmup 8 --profile gpurun_out/comparator_prof.txt > gpurun_out/comparator.log 2>&1
