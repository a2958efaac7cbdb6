import sys, os, torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pytorch_multiprocessing_distributed_amd.models import build_model
from pytorch_multiprocessing_distributed_amd.ops import functional as OF
from pytorch_multiprocessing_distributed_amd.parallel.dp import DataParallel
DEV = "cuda"
for name, stem, hw in [("resnet50", "imagenet", 64), ("res", "cifar", 32), ("resnet50", "cifar", 32)]:
    torch.manual_seed(0)
    nc = 1000 if stem == "imagenet" else 10
    base = build_model(name, num_classes=nc, stem=stem).to(DEV)
    x = torch.randn(4, hw, hw, 8, device=DEV); x[..., 3:] = 0; x = x.to(torch.bfloat16)
    y = torch.randint(0, nc, (4,), device=DEV)
    res = {}
    for mode in ("hip", "torch"):
        m = build_model(name, num_classes=nc, stem=stem).to(DEV); m.load_state_dict(base.state_dict())
        dp = DataParallel(m, None)
        OF.force_torch_prims(mode == "torch")
        dp.zero_grad(); loss = OF.cross_entropy(dp(x), y); loss.backward(); torch.cuda.synchronize()
        OF.force_torch_prims(False)
        res[mode] = (loss.item(), {n: p.grad.float().clone() for n, p in m.named_parameters()})
    print(name, stem, "loss", res["hip"][0], res["torch"][0])
    for k, g in res["torch"][1].items():
        h = res["hip"][1][k]
        cos = torch.nn.functional.cosine_similarity(h.flatten(), g.flatten(), dim=0).item()
        if cos < 0.999: print("   ", k, round(cos, 4), h.norm().item(), g.norm().item())
