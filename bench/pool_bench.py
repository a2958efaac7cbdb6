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

# fused stem tail (BN+ReLU+pool fwd; pool-bwd + BN-bwd reduce / elementwise)
C = x.shape[-1]
p = torch.stack([torch.randn(C, device="cuda") * 0.1, torch.rand(C, device="cuda") + 0.5,
                 torch.randn(C, device="cuda"), torch.randn(C, device="cuda") * 0.5]).contiguous()
so, sarg = HP.stem_pool_fwd(x, p)
gamma = torch.rand(C, device="cuda") + 0.5
red = HP.stats_collapse(HP.stem_pool_bwd_reduce(g, sarg, x, p)).view(2, C)


def sreduce():
    HP._release(HP.stem_pool_bwd_reduce(g, sarg, x, p))


t1 = timeit(lambda: HP.stem_pool_fwd(x, p))
t2 = timeit(sreduce)
t3 = timeit(lambda: HP.stem_pool_bwd_elemt(g, sarg, x, p, gamma, red, float(x.numel() // C)))
yb, ob = x.numel() * 2, so.numel() * 2
print(f"stem pool fwd {t1:.0f} us ({(yb + ob * 2) / t1 / 1e3:.2f} TB/s)  bwd reduce {t2:.0f} us "
      f"({(yb + ob * 2) / t2 / 1e3:.2f} TB/s)  bwd elemt {t3:.0f} us ({(2 * yb + ob * 2) / t3 / 1e3:.2f} TB/s)")
