# Short-reduction wide-output convs (1x1 expand fwd, conv1 dgrad): tile / pipeline variants
set -o pipefail
export PMD_NO_AUTOBUILD=1
for pass in fwd dgrad; do
for sh in "256 14 1024 1 1" "512 7 2048 1 1" "128 28 512 1 1" "64 56 256 1 1"; do
  if [ $pass = dgrad ]; then set -- $sh; sh="$3 $2 $1 $4 $5"; fi
  for cfg in "--tile 1 --impl 7" "--tile 1 --impl 4" "--tile 3 --pipe 0" "--tile 3 --pipe 1" "--tile 3 --pipe 2" "--tile 2 --pipe 0" "--tile 2 --pipe 1" "--tile 2 --pipe 2" "--tile 4" "--tile 5"; do
    timeout -k 5 60 python bench/conv_one.py $sh $cfg --nostats --pass $pass --iters 10 2>/dev/null | grep done || exit 1
  done
done
done
