# PMC counters of every kernel of one command, 3 passes (default command: one full
# ResNet-50 bs256 training step via bench.py).  Each pass stays within the
# per-block counter limits (<= 8 SQ, <= 4 TCC, <= 2 GRBM) and runs alone.
#   bash bench/pmc_step.sh [outdir] [-- command ...]
#   summary: python bench/pmc_summary.py <outdir> [--all]
set -o pipefail
out=${1:-gpurun_out/pmc}; shift || true
[ "${1:-}" = "--" ] && shift
if [ $# -eq 0 ]; then set -- python3 bench.py --steps 2 --warmup 1; fi
mkdir -p "$out"
root=$(pwd)
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$root}"
export PMD_NO_AUTOBUILD=1
PA="SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE"
PB="FETCH_SIZE TCC_HIT_sum GRBM_GUI_ACTIVE"
PC="WRITE_SIZE TCC_MISS_sum GRBM_GUI_ACTIVE"
for p in A B C; do
  eval cnt=\$P$p
  timeout -s KILL 150 rocprofv3 --kernel-trace --pmc $cnt --output-format csv -d "$out/pass$p" -o run -- \
    "$@" > "$out/pass$p.log" 2>&1 || exit 1
done
echo all-ok
