import sys, os, torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pytorch_multiprocessing_distributed_amd.models.resnet import Bottleneck
from pytorch_multiprocessing_distributed_amd.ops import functional as OF, hip_prims as HP, torch_prims as TP
from pytorch_multiprocessing_distributed_amd.parallel.flat import flatten_module
DEV = "cuda"
def run(variant):
    torch.manual_seed(0)
    base = Bottleneck(256, 64, 1).to(DEV)
    x0 = torch.randn(8, 28, 28, 256, device=DEV).to(torch.bfloat16)
    res = {}
    dout = None
    for mode in ("hip", "torch"):
        blk = Bottleneck(256, 64, 1).to(DEV); blk.load_state_dict(base.state_dict())
        if variant != "noflat": flatten_module(blk)
        x = x0.clone().requires_grad_(True)
        OF.force_torch_prims(mode == "torch")
        out = blk(x)
        if dout is None: dout = torch.randn_like(out)
        out.backward(dout); torch.cuda.synchronize()
        OF.force_torch_prims(False)
        res[mode] = (out.float(), x.grad.float())
    d = (res["hip"][1] - res["torch"][1]).abs()
    print(variant, "out err", ((res["hip"][0]-res["torch"][0]).abs().max()/res["torch"][0].abs().max()).item(),
          "dx err", (d.max()/res["torch"][1].abs().max()).item(), "argmax", divmod(d.argmax().item(), 256),
          "n bad", (d > 0.05*res["torch"][1].abs().max()).sum().item())
run("default")
run("noflat")
orig = HP.conv_dgrad
def dg(dy, wpack, x_shape, stride, pad, addend=None):
    r = orig(dy, wpack, x_shape, stride, pad, None)
    return r if addend is None else (r.float() + addend.float()).to(r.dtype)
HP.conv_dgrad = dg
run("unfused_addend")
HP.conv_dgrad = orig
# direct check of dgrad+addend for this shape
torch.manual_seed(1)
w = (torch.randn(64, 256, 1, 1, device=DEV)/16).contiguous(memory_format=torch.channels_last)
wp = HP.conv_weight(w, torch.bfloat16, 256, True); wr = TP.conv_weight(w, torch.bfloat16, 256)
dy = torch.randn(8, 28, 28, 64, device=DEV).to(torch.bfloat16)
add = torch.randn(8, 28, 28, 256, device=DEV).to(torch.bfloat16)
a = HP.conv_dgrad(dy, wp, (8,28,28,256), 1, 0, add).float(); b = TP.conv_dgrad(dy, wr, (8,28,28,256), 1, 0, add).float()
print("dgrad+addend 1x1", ((a-b).abs().max()/b.abs().max()).item())
