"""The HIP-graph training step (engine/train.py GraphedStep) against the eager one-stream step, in
the deterministic statistics mode (ops/functional.py set_deterministic: every statistics
producer's per-block partials folded in a fixed order), where both must agree BIT FOR BIT:

* GraphedStep directly: 5 steps from the same start, the graph captured at step 2 and replayed
  for steps 2-4 with a learning-rate change between replays -> identical parameters, momentum,
  BN running statistics and losses;
* train_epoch in graph mode (the path ``--step_mode auto`` takes for the reference's CIFAR
  workload at W=1): 2 epochs of 4 full batches + a partial last batch (which falls back to an
  eager step after the capture), validate() between the epochs, against the same epochs in
  one_stream mode -> identical state; the captured graph belongs to the optimizer (a second
  model in the same process captures its own);
* negative control: a replay whose captured learning rate is NOT refreshed differs."""
import copy
from types import SimpleNamespace

import pytest
import torch

pytestmark = pytest.mark.gpu


def _state(m, opt):
    return (opt.flat.param_arena.clone(), opt.momentum_arena.clone(),
            torch.cat([v.float().reshape(-1) for k, v in m.module.state_dict().items() if "running" in k]))


@pytest.fixture
def det_one_stream():
    from pytorch_multiprocessing_distributed_amd.models import build_model
    from pytorch_multiprocessing_distributed_amd.ops import functional as OF
    dev = torch.device("cuda", 0)
    OF.init_step_streams(dev)
    OF.set_wgrad_stream(False)
    OF.set_deterministic(True)
    try:
        torch.manual_seed(0)
        yield build_model("res", num_classes=10, stem="cifar").to(dev)
    finally:
        OF.set_deterministic(False)
        OF.set_wgrad_stream(True)


def _steps(mode, m0, batches, stale_lr=False):
    from pytorch_multiprocessing_distributed_amd.engine.optim import FusedSGD
    from pytorch_multiprocessing_distributed_amd.engine.train import GraphedStep
    from pytorch_multiprocessing_distributed_amd.ops import functional as OF
    from pytorch_multiprocessing_distributed_amd.parallel.dp import DataParallel
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
            if stale_lr:
                g.opt.sync_lr = lambda: None      # negative control: the device LR never refreshed
            _, loss = g(x, y)
        else:
            loss = OF.cross_entropy(m(x), y)
            opt.zero_grad()
            loss.backward(OF.loss_seed(loss))
            opt.step()
        losses.append(loss.detach().clone())
    torch.cuda.synchronize()
    assert opt.steps == len(batches)
    return (torch.stack(losses),) + _state(m, opt)


def test_graphed_step_is_bit_exact(det_one_stream):
    from pytorch_multiprocessing_distributed_amd.ops.native import C
    batches = [C.synth_images(32, 32, 32, 8, 3, 10, 7 + s, 0) for s in range(5)]
    _steps("eager", det_one_stream, batches)          # tunes the kernel choices, sizes the scratch
    eager = _steps("eager", det_one_stream, batches)
    eager2 = _steps("eager", det_one_stream, batches)
    graph = _steps("graph", det_one_stream, batches)
    names = ("losses", "params", "momentum", "running")
    for n, a, b in zip(names, eager2, eager):
        assert torch.equal(a, b), f"deterministic mode is not deterministic ({n})"
    for n, a, b in zip(names, graph, eager):
        assert torch.equal(a, b), n
    stale = _steps("graph", det_one_stream, batches, stale_lr=True)
    assert not torch.equal(stale[1], eager[1]), "a stale learning rate went unnoticed"


class _Log:
    def __init__(self):
        self.rows = []

    def write(self, row):
        self.rows.append(row)


def _epochs(mode, m0, batches, epochs=2):
    from pytorch_multiprocessing_distributed_amd.engine.optim import FusedSGD
    from pytorch_multiprocessing_distributed_amd.engine.train import _graph_of, train_epoch, validate
    from pytorch_multiprocessing_distributed_amd.parallel.dp import DataParallel
    dev = torch.device("cuda", 0)
    m = DataParallel(copy.deepcopy(m0), None)
    opt = FusedSGD(m, lr=0.01, momentum=0.9, weight_decay=1e-4, nesterov=True)
    args = SimpleNamespace(step_mode_resolved=mode, print_freq=10 ** 9, compat_metrics=False)
    tr, te = _Log(), _Log()
    for ep in range(epochs):
        opt.param_groups[0]["lr"] = 0.01 * (0.5 ** ep)
        train_epoch(batches, m, opt, ep, tr, args, 0, dev, None, step_offset=ep * len(batches))
        validate(batches[:2], m, ep, te, args, 0, dev, None)
    torch.cuda.synchronize()
    g = _graph_of(opt)
    assert (g is not None) == (mode == "graph")
    return tr.rows, te.rows, _state(m, opt)


def test_train_epochs_graph_mode_with_partial_batch_is_bit_exact(det_one_stream):
    from pytorch_multiprocessing_distributed_amd.ops.native import C
    batches = [C.synth_images(32, 32, 32, 8, 3, 10, 31 + s, 0) for s in range(4)]
    batches.append(C.synth_images(16, 32, 32, 8, 3, 10, 99, 0))     # partial last batch
    _epochs("one_stream", det_one_stream, batches, 1)                # tuning / scratch warm-up
    eager = _epochs("one_stream", det_one_stream, batches)
    graph = _epochs("graph", det_one_stream, batches)
    assert graph[0] == eager[0]          # per-epoch (loss, top-1) rows, bit for bit
    assert graph[1] == eager[1]
    for n, a, b in zip(("params", "momentum", "running"), graph[2], eager[2]):
        assert torch.equal(a, b), n
    again = _epochs("graph", det_one_stream, batches)   # a new optimizer captures its own graph
    for a, b in zip(again[2], eager[2]):
        assert torch.equal(a, b)
