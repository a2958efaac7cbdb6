export PMD_NO_AUTOBUILD=1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
bash bench/gpu_run.sh \
 "fresh:300:python bench.py" \
 "r50:200:python bench.py --steps 30 --warmup 10" \
 "f8:200:python bench.py --steps 30 --warmup 10 --dtype fp8" \
 "r152:300:python bench.py --steps 20 --warmup 8 --model resnet152" \
 "reh:200:python bench.py --steps 30 --warmup 10 --dp_rehearsal" \
 "gputests:900:python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread" \
 "smoke:300:python -c 'import __graft_entry__ as g; g.smoke(); print(\"smoke ok\")'"
