import sys, traceback, torch
sys.path.insert(0, '.')
from pytorch_multiprocessing_distributed_amd.ops import hip_prims as HP
from pytorch_multiprocessing_distributed_amd.models import build_model
from pytorch_multiprocessing_distributed_amd.ops import functional as OF
from pytorch_multiprocessing_distributed_amd.engine.optim import FusedSGD
from pytorch_multiprocessing_distributed_amd.parallel.dp import DataParallel
from pytorch_multiprocessing_distributed_amd.data.loader import SyntheticImageNet
orig = HP._acquire
state = {"on": False}
def acq(c, dev):
    lst = HP._POOL.get((dev, c))
    if state["on"] and not lst:
        print("POOL MISS c=%d" % c)
        traceback.print_stack(limit=6)
    return orig(c, dev)
HP._acquire = acq
dev = torch.device("cuda", 0)
torch.cuda.set_device(0)
m = DataParallel(build_model("resnet50", num_classes=1000, stem="imagenet").to(dev), None)
opt = FusedSGD(m, lr=0.1, momentum=0.9, weight_decay=1e-4, nesterov=True)
data = SyntheticImageNet(64, 224, 1000, steps=6, device=dev, dtype=torch.bfloat16, cpad=8, seed=0)
m.train()
for i in range(5):
    state["on"] = i >= 3
    if state["on"]: print("=== step", i)
    x, y = data.batch_at(i)
    loss = OF.cross_entropy(m(x), y)
    opt.zero_grad(); loss.backward(); opt.step()
torch.cuda.synchronize()
print("done")
