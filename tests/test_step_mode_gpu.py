"""The HIP-graph training step (engine/train.py GraphedStep) against the eager one-stream step: the
same model, batches and optimizer from the same start, 5 steps each (the graph captured at step 2 and
replayed for steps 2-4, a learning-rate change between replays), must end at the same parameters, BN
running statistics and momentum up to the run-to-run noise of the eager step itself (the order of the
statistics atomics): graph-vs-eager within 3x eager-vs-eager."""
import copy

import pytest
import torch

pytestmark = pytest.mark.gpu


def _rel(a, b):
    a, b = a.double(), b.double()
    return ((a - b).norm() / b.norm().clamp_min(1e-30)).item()


def test_graphed_step_matches_eager_one_stream():
    from pytorch_multiprocessing_distributed_amd.engine.optim import FusedSGD
    from pytorch_multiprocessing_distributed_amd.engine.train import GraphedStep
    from pytorch_multiprocessing_distributed_amd.models import build_model
    from pytorch_multiprocessing_distributed_amd.ops import functional as OF
    from pytorch_multiprocessing_distributed_amd.ops.native import C
    from pytorch_multiprocessing_distributed_amd.parallel.dp import DataParallel
    dev = torch.device("cuda", 0)
    OF.init_step_streams(dev)
    OF.set_wgrad_stream(False)
    try:
        torch.manual_seed(0)
        m0 = build_model("res", num_classes=10, stem="cifar").to(dev)
        batches = [C.synth_images(32, 32, 32, 8, 3, 10, 7 + s, 0) for s in range(5)]
        runs = {}
        for mode in ("warm", "eager", "graph", "eager2"):     # "warm": tunes the kernel choices
            m = DataParallel(copy.deepcopy(m0), None)
            m.train()
            opt = FusedSGD(m, lr=0.01, momentum=0.9, weight_decay=1e-4, nesterov=True)
            g = None
            losses = []
            for i, (x, y) in enumerate(batches):
                if i == 3:
                    opt.param_groups[0]["lr"] = 0.005     # a scheduler step between replays
                if mode == "graph" and i == 2:
                    g = GraphedStep(m, opt, x, y)
                if g is not None:
                    _, loss = g(x, y)
                else:
                    loss = OF.cross_entropy(m(x), y)
                    opt.zero_grad()
                    loss.backward(OF.loss_seed(loss))
                    opt.step()
                losses.append(float(loss.detach()))
            torch.cuda.synchronize()
            runs[mode] = (losses, opt.flat.param_arena.clone(), opt.momentum_arena.clone(),
                          torch.cat([v.float().reshape(-1) for k, v in m.module.state_dict().items()
                                     if "running" in k]), opt.steps)
        le, pe, me, be, ne = runs["eager"]
        lg, pg, mg, bg, ng = runs["graph"]
        l2, p2, m2, b2, _ = runs["eager2"]
        assert ne == ng == 5
        for a, b, c in zip(le, lg, l2):
            assert abs(b - a) <= 3 * abs(c - a) + 1e-3 * abs(a), (le, lg, l2)
        for name, x_g, x_e, x_2 in (("params", pg, pe, p2), ("momentum", mg, me, m2), ("running", bg, be, b2)):
            assert _rel(x_g, x_e) <= 3 * _rel(x_2, x_e) + 1e-4, (name, _rel(x_g, x_e), _rel(x_2, x_e))
    finally:
        OF.set_wgrad_stream(True)
