# Mainloop speed-of-light probe: big GEMM-like conv shapes through each tile config
set -o pipefail
export PMD_NO_AUTOBUILD=1
for sh in "1024 28 1024 1 1" "512 28 512 3 1" "256 14 256 3 1" "128 28 128 3 1"; do
  for cfg in "--tile 3 --pipe 0" "--tile 3 --pipe 3" "--tile 2 --pipe 0" "--tile 2 --pipe 1" "--tile 1 --impl 1" "--tile 1 --impl 3" "--tile 1 --impl 6" "--tile 4" "--tile 5"; do
    timeout -k 5 60 python bench/conv_one.py $sh $cfg --nostats --iters 10 2>/dev/null | grep done || exit 1
  done
done
