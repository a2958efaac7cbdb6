# round-5 GPU step 33: step modes -- graph vs eager test, main.py CIFAR with the graph step, bench CIFAR / R50 per mode
set -o pipefail
mkdir -p gpurun_out
export PMD_NO_AUTOBUILD=1
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_step_mode_gpu.py > gpurun_out/t33.log 2>&1 &&
timeout -k 10 300 python main.py --world_size 1 --synthetic --train_samples 4096 --epochs 2 --save_path gpurun_out/m33 --no_plot > gpurun_out/m33.log 2>&1 &&
O=gpurun_out/step_modes.jsonl && : > $O &&
for m in two_stream one_stream graph; do
  timeout -k 10 200 python bench.py --model res --stem cifar --batch 32 --image 32 --classes 10 --steps 300 --warmup 20 --step_mode $m 2>/dev/null | tail -1 >> $O || exit 1
done &&
timeout -k 10 200 python bench.py --step_mode one_stream 2>/dev/null | tail -1 >> $O &&
timeout -k 10 200 python bench.py 2>/dev/null | tail -1 >> $O
