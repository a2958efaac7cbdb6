# PMC passes on one conv layer (C256 14x14 K256 3x3 fwd) for each tile config.
set -o pipefail
mkdir -p gpurun_out/pmc
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export PMD_NO_AUTOBUILD=1
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU"
P2="SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_VMEM SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_WAIT_INST_ANY SQ_INST_LEVEL_VMEM TCC_HIT_sum TCC_MISS_sum"
for cfg in "t1i1:--tile 1 --impl 1" "t1i4:--tile 1 --impl 4" "t3p0:--tile 3 --pipe 0" "t2p1:--tile 2 --pipe 1"; do
  name=${cfg%%:*}; args=${cfg#*:}
  timeout -s KILL 60 rocprofv3 --pmc $P1 --output-format csv -d gpurun_out/pmc/${name}_p1 -o run -- python3 bench/conv_one.py 256 14 256 3 1 $args --iters 10 > gpurun_out/pmc/${name}_p1.log 2>&1 || exit 1
  timeout -s KILL 60 rocprofv3 --pmc $P2 --output-format csv -d gpurun_out/pmc/${name}_p2 -o run -- python3 bench/conv_one.py 256 14 256 3 1 $args --iters 10 > gpurun_out/pmc/${name}_p2.log 2>&1 || exit 1
done
echo all-ok
