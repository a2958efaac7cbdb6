# P8 pipeline vs the existing tile configs on MFMA-heavy conv shapes (fwd and dgrad, no stats)
set -o pipefail
export PMD_NO_AUTOBUILD=1
for pass in fwd dgrad; do
for sh in "1024 28 1024 1 1" "256 14 256 3 1" "128 28 128 3 1" "512 7 512 3 1" "64 56 64 3 1" "1024 14 256 1 1"; do
  for cfg in "--tile 3 --pipe 0" "--tile 2 --pipe 0" "--tile 1 --impl 1" "--tile 4" "--tile 6" "--tile 7" "--tile 8" "--tile 9"; do
    timeout -k 5 60 python bench/conv_one.py $sh $cfg --nostats --pass $pass --iters 10 2>/dev/null | grep done || exit 1
  done
done
done
