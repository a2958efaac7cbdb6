"""The native fork/join event ring (csrc/runtime/events.cpp) that can carry the training step's
main <-> weight-gradient stream hand-offs (ops/functional.py PMD_FORK_EVENTS):

* exactness of both hand-off directions in every fence mode: main writes a 4 KB / 64 MB buffer ->
  fork -> the side stream reads it; the side stream writes -> join -> main reads, 200 rounds on
  double buffers (a stale line in any XCD's L2 would show as a wrong value);
* the two-stream ResNet-18-ref backward with its fork / join points on the ring (no system
  fence) gives BIT-IDENTICAL parameter gradients, BN running statistics and losses to the same
  backward on torch's events, in the deterministic statistics mode (ops/functional.py
  set_deterministic: private per-block statistic slots folded in a fixed order), with and
  without the main stream held back so the side stream really waits at every fork;
* negative control: the same comparison with ONE fork dropped (the side stream reads dY before
  the main stream has produced it) must fail."""
import copy

import pytest
import torch

pytestmark = pytest.mark.gpu


def _rel(a, b):
    a, b = a.double(), b.double()
    return ((a - b).norm() / b.norm().clamp_min(1e-30)).item()


@pytest.mark.parametrize("n", [1024, 16 << 20])
@pytest.mark.parametrize("mode", [0, 1, 2])
def test_ring_handoffs_exact(mode, n):
    """n = 1024: 4 KB buffers re-read every round with no other traffic in between, so a
    stale line left in the reading XCD's L2 (or CU L1) would survive to the next read."""
    from pytorch_multiprocessing_distributed_amd.ops.native import C
    dev = torch.device("cuda", 0)
    main = torch.cuda.current_stream(dev)
    side = torch.cuda.Stream(device=dev)
    ring = C.StreamEvents(64, mode, 0)
    assert ring.mode == mode
    iters = 200
    idx = torch.arange(0, n, 4099 if n > 4096 else 1, device=dev)
    bufs = [torch.zeros(n, device=dev) for _ in range(2)]
    back = [torch.zeros(n, device=dev) for _ in range(2)]
    got_side = torch.zeros(iters, device=dev)
    got_main = torch.zeros(iters, device=dev)
    hm, hs = main.cuda_stream, side.cuda_stream
    for i in range(iters):
        b, r = bufs[i % 2], back[i % 2]
        b.fill_(float(i))
        ring.fork(hm, hs)
        with torch.cuda.stream(side):
            got_side[i] = b[idx].min() + b[idx].max() - float(i)
            r.fill_(float(i) + 0.5)
        slot = ring.record(hs)
        ring.wait(hm, slot)
        got_main[i] = r[idx].min() + r[idx].max() - float(i) - 1.0
    torch.cuda.synchronize()
    want = torch.arange(iters, device=dev, dtype=torch.float32)
    assert torch.equal(got_side, want)
    assert torch.equal(got_main, want)
    assert ring.records == 2 * iters
    assert ring.query(slot)


def _grads(mode, m0, batches, lag_us=0, drop=-1):
    """Per-tensor parameter gradients (+ running statistics, losses) of one backward per batch
    (no optimizer step) on the two-stream schedule, the hand-offs on torch events (mode -1) or
    the native ring (mode >= 0).  lag_us: the main stream idles that long before each
    backward, so every fork is taken while the side stream's work is ahead of its producer;
    drop >= 0: the fork with that index in each backward is skipped (negative control)."""
    from pytorch_multiprocessing_distributed_amd.engine.optim import FusedSGD
    from pytorch_multiprocessing_distributed_amd.ops import functional as OF
    from pytorch_multiprocessing_distributed_amd.ops.native import C
    from pytorch_multiprocessing_distributed_amd.parallel.dp import DataParallel
    OF._FORK_EV = mode
    OF._RINGS.clear()
    m = DataParallel(copy.deepcopy(m0), None)
    m.train()
    opt = FusedSGD(m, lr=0.01, momentum=0.9, weight_decay=1e-4, nesterov=True)
    grads, losses = [], []
    try:
        for x, y in batches:
            loss = OF.cross_entropy(m(x), y)
            opt.zero_grad()
            if lag_us:
                C.gpu_sleep(lag_us)
            OF._DROP_FORK[0] = drop
            loss.backward(OF.loss_seed(loss))
            OF._DROP_FORK[0] = -1
            torch.cuda.synchronize()
            g = opt.flat.grad_arena
            grads += [g[o:o + p.numel()].clone() for p, o in zip(opt.flat.params, opt.flat.offsets)]
            losses.append(loss.detach().clone())
        if mode >= 0:
            ring = OF._RINGS[batches[0][0].device]
            assert ring.mode == mode and ring.records > 5 * len(batches)   # the step used the ring
    finally:
        OF._DROP_FORK[0] = -1
        OF._RINGS.clear()
    running = [v.clone() for k, v in m.module.state_dict().items() if "running" in k]
    return grads, running, losses


def _differences(a, b):
    return [i for i, (x, y) in enumerate(zip(a, b)) if not torch.equal(x, y)]


@pytest.fixture
def det_two_stream(monkeypatch):
    from pytorch_multiprocessing_distributed_amd.models import build_model
    from pytorch_multiprocessing_distributed_amd.ops import functional as OF
    from pytorch_multiprocessing_distributed_amd.ops.native import C
    dev = torch.device("cuda", 0)
    OF.init_step_streams(dev)
    OF.set_wgrad_stream(True)
    monkeypatch.setattr(OF, "_FORK_EV", OF._FORK_EV)
    OF.set_deterministic(True)
    try:
        torch.manual_seed(0)
        m0 = build_model("res", num_classes=10, stem="cifar").to(dev)
        batches = [C.synth_images(32, 32, 32, 8, 3, 10, 11 + s, 0) for s in range(3)]
        _grads(-1, m0, batches)            # tunes the kernel choices, sizes the scratch
        yield m0, batches
    finally:
        OF.set_deterministic(False)


@pytest.mark.parametrize("lag_us", [0, 20000])
def test_two_stream_step_on_ring_is_bit_exact(det_two_stream, lag_us):
    m0, batches = det_two_stream
    ref = _grads(-1, m0, batches)
    again = _grads(-1, m0, batches, lag_us)
    # the deterministic mode itself: two torch-event runs agree bit for bit
    for a, b in zip(ref, again):
        assert not _differences(a, b), "deterministic mode is not deterministic"
    for mode in (0, 1, 2):
        got = _grads(mode, m0, batches, lag_us)
        for what, a, b in zip(("grads", "running", "losses"), got, ref):
            bad = _differences(a, b)
            assert not bad, (mode, what, bad[:10])


def test_dropped_fork_is_caught(det_two_stream):
    """Negative control: the first fork of every backward skipped (its weight gradient reads dY
    while the main stream is still held back) -- the bit-exact oracle must see it."""
    m0, batches = det_two_stream
    ref = _grads(-1, m0, batches)
    got = _grads(1, m0, batches, lag_us=20000, drop=0)
    assert _differences(got[0], ref[0]), "a dropped fork went unnoticed"
    # the control breaks only the weight gradient it hands off: the main-stream state agrees
    assert not _differences(got[1], ref[1])


def test_side_stream_shortcut_is_bit_exact(det_two_stream, monkeypatch):
    """The forward's projection-shortcut convs on the side stream (concurrent with the main path,
    joined before the final BN-apply) == the same step with them on the main stream, bit for bit
    (gradients, running statistics, losses), with the main stream held back so the side stream
    really runs ahead."""
    from pytorch_multiprocessing_distributed_amd.ops import functional as OF
    m0, batches = det_two_stream
    monkeypatch.setattr(OF, "_SIDE_SHORTCUT", False)
    ref = _grads(1, m0, batches)
    monkeypatch.setattr(OF, "_SIDE_SHORTCUT", True)
    for lag in (0, 20000):
        got = _grads(1, m0, batches, lag)
        for what, a, b in zip(("grads", "running", "losses"), got, ref):
            bad = _differences(a, b)
            assert not bad, (lag, what, bad[:10])
