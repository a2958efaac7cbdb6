"""AddressSanitizer over the framework's host C++: the binding
layer and the native runtime -- the bucketed gradient reducer (mark / ordered
launch / finalize / ready-order rebuild / bf16 wire buffers), the tuning-table
import/export -- built with ``-Xarch_host -fsanitize=address`` (device code is
never sanitised; csrc/build.py --asan) and driven by a 2-rank gloo training run
on the CPU with the ASan runtime preloaded.  Any heap/stack/use-after-free
error aborts the run with an AddressSanitizer report."""
import os
import socket
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

SCRIPT = r"""
import datetime, os, sys
import torch, torch.distributed as dist, torch.multiprocessing as mp
sys.path.insert(0, %(root)r)

def worker(rank, world):
    dist.init_process_group("gloo", rank=rank, world_size=world, timeout=datetime.timedelta(seconds=120))
    from pytorch_multiprocessing_distributed_amd.ops.native import C
    assert "asan" in C.__file__, C.__file__
    from pytorch_multiprocessing_distributed_amd.engine.optim import FusedSGD
    from pytorch_multiprocessing_distributed_amd.models import build_model
    from pytorch_multiprocessing_distributed_amd.ops import functional as OF
    from pytorch_multiprocessing_distributed_amd.parallel.comm import get_comm
    from pytorch_multiprocessing_distributed_amd.parallel.dp import DataParallel
    torch.manual_seed(0)
    comm = get_comm()
    OF.set_bn_sync(comm)
    for compress in ("none", "bf16"):
        dp = DataParallel(build_model("res"), comm, bucket_mb=0.25, first_bucket_mb=0.05,
                          compress=compress, timeline=True)
        opt = FusedSGD(dp, lr=0.05)
        x = torch.randn(4, 32, 32, 8)
        y = torch.arange(4) %% 10
        for step in range(4):
            ctx = dp.no_sync() if step == 2 else torch.enable_grad()
            with ctx:
                loss = OF.cross_entropy(dp(x), y)
                opt.zero_grad()
                loss.backward()
            opt.step()
        assert dp.num_iterations == 3, dp.num_iterations
        assert dp.rebuilt_order is not None
        dp.bucket_timeline()
        dp.close()
    C.conv_autotune_import(C.conv_autotune_export())
    OF.set_bn_sync(None)
    dist.destroy_process_group()

if __name__ == "__main__":
    mp.spawn(worker, args=(2,), nprocs=2, join=True)
    print("asan-run-ok")
"""


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.slow
def test_native_runtime_under_asan(tmp_path):
    sys.path.insert(0, os.path.join(ROOT, "csrc"))
    try:
        import build as B
    finally:
        sys.path.pop(0)
    rt = B.asan_runtime()
    if rt is None:
        pytest.skip("no clang ASan runtime in this toolchain")
    B.build(asan=True, verbose=False)
    script = tmp_path / "asan_run.py"
    script.write_text(SCRIPT % {"root": ROOT})
    env = dict(os.environ, LD_PRELOAD=rt, PMD_EXT_DIR=B.ASAN_DIR, MASTER_ADDR="127.0.0.1",
               MASTER_PORT=str(_port()), PMD_NO_AUTOBUILD="1",
               ASAN_OPTIONS="detect_leaks=0:halt_on_error=1:detect_odr_violation=0")
    r = subprocess.run([sys.executable, str(script)], env=env, capture_output=True, text=True,
                       timeout=900, cwd=ROOT)
    report = r.stdout[-4000:] + r.stderr[-4000:]
    assert "AddressSanitizer" not in r.stderr, report
    assert r.returncode == 0 and "asan-run-ok" in r.stdout, report
