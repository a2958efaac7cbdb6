# HALO 3x3 conv (tile policy 11) vs the autotuned-equivalent configs on the 3x3 stride-1 layers
set -o pipefail
export PMD_NO_AUTOBUILD=1
for pass in fwd dgrad; do
for sh in "64 56 64 3 1" "128 28 128 3 1" "256 14 256 3 1" "512 7 512 3 1"; do
  for cfg in "--tile 11" "--tile 12" "--tile 1 --impl 1" "--tile 1 --impl 7" "--tile 3 --pipe 0" "--tile 4"; do
    timeout -k 5 60 python bench/conv_one.py $sh $cfg --nostats --pass $pass --iters 10 2>/dev/null | grep done || exit 1
  done
done
done
