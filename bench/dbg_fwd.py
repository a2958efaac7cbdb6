import sys, os, torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pytorch_multiprocessing_distributed_amd.models import build_model
from pytorch_multiprocessing_distributed_amd.ops import functional as OF
from pytorch_multiprocessing_distributed_amd.ops import hip_prims as HP, torch_prims as TP
DEV = "cuda"
torch.manual_seed(0)
m = build_model("resnet50", num_classes=10, stem="cifar").to(DEV)
x = torch.randn(4, 32, 32, 8, device=DEV); x[..., 3:] = 0; x = x.to(torch.bfloat16)
outs = {}
def hook(name):
    def f(mod, inp, out): outs.setdefault(name, []).append(out.detach().float().clone())
    return f
for n, mod in m.named_modules():
    if n.count('.') == 1 and n.startswith('layer'): mod.register_forward_hook(hook(n))
for mode in ("hip", "torch"):
    OF.force_torch_prims(mode == "torch")
    with torch.no_grad():
        m.train()
        m(x)
OF.force_torch_prims(False)
for k, (a, b) in outs.items():
    print(k, ((a - b).norm() / b.norm()).item())
# single block, isolated: run layer1.1 on the same input with both prims
blk = m.layer1[1]
inp = torch.randn(4, 32, 32, 256, device=DEV).to(torch.bfloat16)
r = {}
for mode in ("hip", "torch"):
    OF.force_torch_prims(mode == "torch")
    with torch.no_grad():
        r[mode] = blk(inp).float()
OF.force_torch_prims(False)
print("layer1.1 isolated", ((r['hip'] - r['torch']).norm() / r['torch'].norm()).item())
# pieces of the identity block
w = blk.conv1.weight
wp = HP.conv_weight(w, torch.bfloat16, 256, True); wr = TP.conv_weight(w, torch.bfloat16, 256)
y, st = HP.conv_fwd(inp, wp, 1, 0, True); yr, sr = TP.conv_fwd(inp, wr, 1, 0, True)
print("conv1", ((y.float()-yr.float()).norm()/yr.float().norm()).item())
flat = HP.stats_collapse(st); print("stats", ((flat.view(2,-1)-sr).norm()/sr.norm()).item())
y, st = HP.conv_fwd(inp, wp, 1, 0, True)
bn = blk.bn1
p = HP.stats_finalize_local(st, float(y.numel()//y.shape[-1]), bn.weight, bn.bias, bn.eps)
pr = TP.stats_finalize_local(sr, float(y.numel()//y.shape[-1]), bn.weight, bn.bias, bn.eps)
print("params", ((p-pr).norm()/pr.norm()).item(), p[:, :4], pr[:, :4])
