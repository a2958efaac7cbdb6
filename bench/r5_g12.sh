# round-5 GPU step 12: kernel traces of the BN fold variants (lin = fold off, fold, folda = fold on every block)
set -o pipefail
mkdir -p gpurun_out
export PMD_NO_AUTOBUILD=1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for v in "lin:PMD_BNFOLD=0" "fold:PMD_BNFOLD=1" "folda:PMD_BNLIN=all"; do
  name=${v%%:*}; envs=${v#*:}
  env $envs timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/kt_$name -o run -- \
    python3 bench.py --steps 16 --warmup 6 > gpurun_out/kt_$name.log 2>&1 || exit 1
done
echo done
