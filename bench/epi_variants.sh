# dgrad-epilogue bench per prebuilt variant (abso/so_<v>.so)
set -o pipefail
export PMD_NO_AUTOBUILD=1
SO=pytorch_multiprocessing_distributed_amd/_C.cpython-310-x86_64-linux-gnu.so
cp $SO abso/so_current_backup.so
for v in "$@"; do
  cp abso/so_$v.so $SO
  echo "== $v"
  timeout -k 10 120 python bench/dgrad_epi_bench.py 2>/dev/null | tail -1 || exit 1
done
cp abso/so_current_backup.so $SO
