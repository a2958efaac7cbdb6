# round-5 GPU step 25: 48 KB weight-gradient variant (32-row x3 DMA) for the tuned 64 KB choices (co-residency A/B)
set -o pipefail
mkdir -p gpurun_out
export PMD_NO_AUTOBUILD=1
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_kernels_gpu.py -k "wgrad" > gpurun_out/t25.log 2>&1 &&
AB_ROUNDS=2 bash bench/ab_env.sh "base:" "m1to7:PMD_WGRAD_MAP1=7" "m0to7:PMD_WGRAD_MAP0=7" "m01to7:PMD_WGRAD_MAP0=7,PMD_WGRAD_MAP1=7" "m4to7:PMD_WGRAD_MAP4=7" > gpurun_out/ab_w7.txt 2>&1
