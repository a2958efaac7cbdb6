# LDS-conflict counters (pass A of bench/pmc_step.sh only) of one ResNet-50 step for each prebuilt
# extension variant abso/so_<name>.so ("base" = the in-tree library):  bash bench/pmc_lds.sh base v1 v2
set -o pipefail
mkdir -p gpurun_out
export PMD_NO_AUTOBUILD=1 PMD_ALLOW_VARIANT=1
SO=pytorch_multiprocessing_distributed_amd/_C.cpython-310-x86_64-linux-gnu.so
cp $SO abso/so_base.so
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
PA="SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE"
for v in "$@"; do
  cp abso/so_$v.so $SO
  timeout -s KILL 150 rocprofv3 --kernel-trace --pmc $PA --output-format csv -d gpurun_out/lds_$v/passA -o run -- \
    python3 bench.py --steps 2 --warmup 1 > gpurun_out/lds_$v.log 2>&1 || { cp abso/so_base.so $SO; exit 1; }
done
cp abso/so_base.so $SO
echo all-ok
