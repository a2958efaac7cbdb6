set -o pipefail
export PMD_NO_AUTOBUILD=1
for sh in "64 56 256 1 1" "128 28 512 1 1" "256 14 1024 1 1" "512 7 2048 1 1" "256 56 64 1 1" "1024 14 256 1 1"; do
  for cfg in "--tile 1 --impl 7" "--tile 1 --impl 7 --nostats" "--tile 1 --impl 4" "--tile 1 --impl 4 --nostats"; do
    timeout -k 5 60 python bench/conv_one.py $sh $cfg --iters 12 || exit 1
  done
done
