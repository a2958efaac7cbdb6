# PMC step profile for two prebuilt variants (abso/so_<a>.so, abso/so_<b>.so)
set -o pipefail
SO=pytorch_multiprocessing_distributed_amd/_C.cpython-310-x86_64-linux-gnu.so
cp $SO abso/so_current_backup.so
for v in "$@"; do
  cp abso/so_$v.so $SO
  bash bench/pmc_step.sh > gpurun_out/pmcstep_$v.log 2>&1 || exit 1
  mv gpurun_out/pmc gpurun_out/pmc_$v
done
cp abso/so_current_backup.so $SO
