import os, sys, socket, torch, torch.multiprocessing as mp
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

def port():
    s = socket.socket(); s.bind(("127.0.0.1", 0)); p = s.getsockname()[1]; s.close(); return p

def run(rank, world, pt, out, sync_bn, model_name):
    import torch.distributed as dist
    from pytorch_multiprocessing_distributed_amd.models import build_model
    from pytorch_multiprocessing_distributed_amd.ops import functional as OF
    from pytorch_multiprocessing_distributed_amd.parallel.comm import get_comm
    from pytorch_multiprocessing_distributed_amd.parallel.dp import DataParallel
    from pytorch_multiprocessing_distributed_amd.ops.native import C
    torch.cuda.set_device(0)
    comm = None
    if world > 1:
        os.environ["MASTER_ADDR"] = "127.0.0.1"; os.environ["MASTER_PORT"] = str(pt)
        dist.init_process_group("gloo", rank=rank, world_size=world)
        comm = get_comm()
        OF.set_bn_sync(comm if sync_bn else None)
    torch.manual_seed(0)
    m = build_model(model_name).cuda()
    acts = {}
    for n, mod in m.named_modules():
        if n in ("layer1", "layer2", "layer3", "layer4", "bn1"):
            mod.register_forward_hook(lambda mod, i, o, n=n: acts.__setitem__(n, o.detach().float().cpu()))
    x, _ = C.synth_images(8, 32, 32, 8, 3, 10, 11, 0)
    y = torch.arange(8, device="cuda") % 10
    per = 8 // world
    xs, ys = x[rank*per:(rank+1)*per], y[rank*per:(rank+1)*per]
    dp = DataParallel(m, comm if os.environ.get("DBG_DP", "1") == "1" else None)
    dp.zero_grad()
    logits = dp(xs)
    loss = OF.cross_entropy(logits, ys)
    loss.backward(); torch.cuda.synchronize()
    if world > 1 and os.environ.get("DBG_DP", "1") == "0":
        for p_ in m.parameters():
            g_ = p_.grad.detach().clone(); dist.all_reduce(g_); p_.grad.copy_(g_ / world)
    if rank == 0:
        torch.save({"acts": {k: v[:per] for k, v in acts.items()}, "logits": logits.detach().float().cpu()[:per],
                    "grads": {n: p.grad.float().cpu() for n, p in m.named_parameters()}}, out)
    if world > 1: dist.destroy_process_group()

if __name__ == "__main__":
  for dbg_dp in ("0", "1"):
    os.environ["DBG_DP"] = dbg_dp
    print("==== reducer in DataParallel:", dbg_dp)
    for model_name in ("res",):
        mp.spawn(run, args=(2, port(), "/tmp/two.pt", True, model_name), nprocs=2, join=True)
        run(0, 1, 0, "/tmp/one.pt", True, model_name)
        a, b = torch.load("/tmp/two.pt"), torch.load("/tmp/one.pt")
        for k in a["acts"]:
            bb = b["acts"][k][:4]; print(model_name, "act", k, ((a["acts"][k] - bb).norm() / bb.norm()).item())
        print("logits", ((a["logits"] - b["logits"][:4]).norm() / b["logits"][:4].norm()).item())
        for n in a["grads"]:
            print("grad", n, ((a["grads"][n] - b["grads"][n]).norm() / b["grads"][n].norm()).item())
