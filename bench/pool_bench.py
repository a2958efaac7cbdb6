"""Max-pool 3x3/s2 (ImageNet stem) fwd/bwd bandwidth at the R50 shape."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pytorch_multiprocessing_distributed_amd.ops import hip_prims as HP  # noqa: E402


def timeit(fn, iters=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(iters):
        fn()
    b.record()
    b.synchronize()
    return a.elapsed_time(b) / iters * 1e3


x = torch.randn(256, 112, 112, 64, device="cuda").to(torch.bfloat16)
out, idx = HP.maxpool_fwd(x)
g = torch.randn_like(out)
tf = timeit(lambda: HP.maxpool_fwd(x))
tb = timeit(lambda: HP.maxpool_bwd(g, idx, tuple(x.shape)))
gb = x.numel() * 2 / 1e9
print(f"maxpool fwd {tf:.0f} us ({(x.numel() * 2 + out.numel() * 3) / tf / 1e3:.2f} TB/s)  "
      f"bwd {tb:.0f} us ({(x.numel() * 2 + out.numel() * 3) / tb / 1e3:.2f} TB/s)")
