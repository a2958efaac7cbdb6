import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pytorch_multiprocessing_distributed_amd.models.resnet import Bottleneck  # noqa: E402
from pytorch_multiprocessing_distributed_amd.ops import functional as OF, hip_prims as HP  # noqa: E402
from pytorch_multiprocessing_distributed_amd.ops.fp8 import Fp8Scaling  # noqa: E402
from pytorch_multiprocessing_distributed_amd.parallel.flat import flatten_module  # noqa: E402

DEV = "cuda"
torch.manual_seed(0)
x = torch.relu(torch.randn(16, 16, 16, 256, device=DEV)).to(torch.bfloat16)
# stats check of the fp8 conv
w = (torch.randn(64, 256, 1, 1, device=DEV) / 16).contiguous(memory_format=torch.channels_last)
f8 = Fp8Scaling(DEV)
sx, ax = f8.site("x")
sw, aw = f8.site("w", init_from=w)
xq = HP.quant_bf16_fp8(x, sx, ax)
wq = HP.quant_weight_fp8(w, 256, sw, aw)
y, st = HP.conv_fp8_fwd(xq, wq, sx, sw, 1, 0, True)
col = HP.stats_collapse(st).view(2, -1)
yf = y.float().reshape(-1, 64)
print("stats sum err", ((col[0] - yf.sum(0)).abs().max() / yf.sum(0).abs().max()).item(),
      "sumsq err", ((col[1] - (yf * yf).sum(0)).abs().max() / (yf * yf).sum(0).max()).item())
# block-level train-mode forward + backward, fp8 vs bf16
base = Bottleneck(256, 64, 1).to(DEV)
sd = base.state_dict()
res = {}
for mode in ("bf16", "fp8"):
    blk = Bottleneck(256, 64, 1).to(DEV)
    blk.load_state_dict(sd)
    flatten_module(blk)
    OF.set_fp8(Fp8Scaling(DEV) if mode == "fp8" else None)
    xi = x.clone().requires_grad_(True)
    out = blk(xi)
    g = torch.randn_like(out, generator=torch.Generator(DEV).manual_seed(1))
    out.backward(g)
    res[mode] = (out.float(), xi.grad.float(), {n: p.grad.float().clone() for n, p in blk.named_parameters()},
                 {k: v.float().clone() for k, v in blk.state_dict().items() if "running" in k})
    OF.set_fp8(None)
a, b = res["fp8"], res["bf16"]
print("out rel", ((a[0] - b[0]).norm() / b[0].norm()).item(), "dx rel", ((a[1] - b[1]).norm() / b[1].norm()).item())
for n in b[2]:
    print("grad", n, ((a[2][n] - b[2][n]).norm() / b[2][n].norm()).item())
for n in b[3]:
    print("buf", n, ((a[3][n] - b[3][n]).norm() / b[3][n].norm().clamp_min(1e-9)).item())
