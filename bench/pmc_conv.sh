# PMC passes on ONE conv layer for several kernel configs (one run per pass per
# config, each under its own limit).  Summarise with bench/pmc_conv_summary.py.
#   bash bench/pmc_conv.sh "C H K R stride" fwd|dgrad "name:conv_one args" ...
set -o pipefail
shape="$1"; which="$2"; shift 2
mkdir -p gpurun_out/pmcc
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export PMD_NO_AUTOBUILD=1
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE"
P2="SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_VALU SQ_INSTS_VMEM SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_INST_LEVEL_VMEM SQ_ACTIVE_INST_VMEM TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE"
tag=$(echo "$shape $which" | tr ' ' '_')
for cfg in "$@"; do
  name=${cfg%%:*}; args=${cfg#*:}
  for p in 1 2; do
    eval cnt=\$P$p
    timeout -s KILL 60 rocprofv3 --kernel-trace --pmc $cnt --output-format csv -d gpurun_out/pmcc/${tag}/${name}_p$p -o run -- \
      python3 bench/conv_one.py $shape --pass $which $args --iters 8 > gpurun_out/pmcc/${tag}_${name}_p$p.log 2>&1 || exit 1
  done
done
echo all-ok
