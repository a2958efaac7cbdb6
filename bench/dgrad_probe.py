"""Per-section time of the data-gradient convolutions inside the ResNet-50 bs256 training step
(where the fused dgrad's time goes).

Needs the timing-only probe build (kernels/conv_igemm.hip PMD_DGRAD_PROBE): every dgrad block's
wave 0 stamps (s_memtime) entry, main loop done, C tile staged, epilogue rows done (after its
stores landed), fused BN-reduce done, plus the wall clock at entry / exit.  One step after the
warmup runs with the probe buffer armed; the records are grouped into launches (the dgrads run
in stream order on the main stream: sorted by entry time, a launch ends where a block enters
after every earlier block exited) and each launch's wall time is split over the sections in
proportion to its blocks' cycles in them.

    PMD_EXTRA_CFLAGS=-DPMD_DGRAD_PROBE=1 python csrc/build.py --variant probe
    bash bench/dgrad_probe.sh [--step_mode one_stream|two_stream] [--dtype bf16|fp8]
"""
import argparse
import collections
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

SECTIONS = ("mainloop", "C staging", "epilogue rows", "BN reduce")


def run(a):
    from pytorch_multiprocessing_distributed_amd.data.loader import SyntheticImageNet
    from pytorch_multiprocessing_distributed_amd.engine.optim import FusedSGD
    from pytorch_multiprocessing_distributed_amd.models import build_model
    from pytorch_multiprocessing_distributed_amd.ops import functional as OF
    from pytorch_multiprocessing_distributed_amd.ops import tuning
    from pytorch_multiprocessing_distributed_amd.ops.native import C
    from pytorch_multiprocessing_distributed_amd.parallel.dp import DataParallel

    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    OF.init_step_streams(dev)
    OF.set_wgrad_stream(a.step_mode == "two_stream")
    torch.manual_seed(0)
    model = DataParallel(build_model("resnet50", num_classes=1000, stem="imagenet").to(dev), None)
    if a.dtype == "fp8":
        from pytorch_multiprocessing_distributed_amd.ops.fp8 import Fp8Scaling
        OF.set_fp8(Fp8Scaling(dev))
    opt = FusedSGD(model, lr=0.1, momentum=0.9, weight_decay=1e-4, nesterov=True)
    data = SyntheticImageNet(a.batch, 224, 1000, steps=a.warmup + 1, device=dev, dtype=torch.bfloat16,
                             cpad=8, seed=0)
    tuning.load_default()
    model.train()

    def step(i):
        x, y = data.batch_at(i)
        loss = OF.cross_entropy(model(x), y)
        opt.zero_grad()
        loss.backward(OF.loss_seed(loss))
        opt.step()

    for i in range(a.warmup):
        step(i)
    torch.cuda.synchronize()

    def timed(i):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        step(i)
        e1.record()
        e1.synchronize()
        return e0.elapsed_time(e1)
    off_ms = sorted(timed(i % a.warmup) for i in range(5))[2]
    buf = torch.zeros(a.cap, 16, dtype=torch.int64, device=dev)
    if C.conv_probe_set(buf) != 1:
        raise SystemExit("not a probe build (PMD_EXTRA_CFLAGS=-DPMD_DGRAD_PROBE=1 python csrc/build.py --variant probe)")
    on_ms = timed(a.warmup)
    n = C.conv_probe_count()
    C.conv_probe_set(torch.zeros(1, 16, dtype=torch.int64, device=dev)[:0])
    if n > a.cap // 256:
        raise SystemExit(f"a probe counter overflowed ({n} > {a.cap // 256} records)")
    recs = buf[buf[:, 0] != 0].cpu().numpy().astype(np.uint64)
    print(f"# step time (events): {off_ms:.3f} ms without records, {on_ms:.3f} ms with them (probe build)")
    return recs


def analyse(recs, label):
    # launches: the dgrads run in stream order (one stream), so sorted by entry time a new launch
    # starts at the first block that enters after every earlier block has exited
    recs = recs[np.argsort(recs[:, 0], kind="stable")]
    launches, cur, end = [], [], 0
    for r in recs:
        r = [int(v) for v in r]
        if cur and r[0] > end:
            launches.append(cur)
            cur = []
        cur.append(r)
        end = max(end, r[1]) if len(cur) > 1 else r[1]
    if cur:
        launches.append(cur)
    launches = [((rs[0][7], rs[0][8], rs[0][9]), rs) for rs in launches]
    mixed = sum(1 for k, rs in launches if any((r[7], r[8], r[9]) != k for r in rs))
    fam = collections.OrderedDict()
    for key, rs in launches:
        wall_us = (max(r[1] for r in rs) - min(r[0] for r in rs)) / 100.0   # 100 MHz wall clock
        cyc = [0, 0, 0, 0]
        for r in rs:
            t = r[2:7]
            for k in range(4):
                cyc[k] += max(t[k + 1] - t[k], 0)
        tot = max(sum(cyc), 1)
        blk_wall = sum((r[1] - r[0]) / 100.0 for r in rs)
        M, Nout, Kg = key[0] >> 32, (key[0] >> 16) & 0xFFFF, key[0] & 0xFFFF
        BM, BN, BK, fl = key[1] >> 48, (key[1] >> 32) & 0xFFFF, (key[1] >> 16) & 0xFFFF, key[1] & 0xFFFF
        stride, nw, nbn, add = key[2] >> 32, (key[2] >> 16) & 0xFF, (key[2] >> 8) & 0xFF, key[2] & 1
        tile = f"{BM}x{BN}x{BK}/{fl >> 8 & 0xFF}st{'/f8' if fl & 16 else ''}{'/1st' if fl & 32 else ''}" \
               f"{'/halo' if fl & 64 else ''}{'/p8' if fl & 128 else ''}/{nw}w"
        shape = f"M={M} C={Nout} K={Kg} s{stride} nbn={nbn} add={add}"
        f = fam.setdefault((tile, shape), {"calls": 0, "wall": 0.0, "sec": [0.0] * 4, "blocks": 0,
                                           "blk_wall": 0.0})
        f["calls"] += 1
        f["wall"] += wall_us
        f["blocks"] += len(rs)
        f["blk_wall"] += blk_wall
        for k in range(4):
            f["sec"][k] += wall_us * cyc[k] / tot
    rows = sorted(fam.items(), key=lambda kv: -kv[1]["wall"])
    total = sum(v["wall"] for _, v in rows)
    print(f"# {label}: {len(launches)} dgrad launches ({mixed} with mixed shapes: must be 0), "
          f"{total / 1000:.3f} ms wall (probe build: each wave drains its stores before the last two stamps)")
    print(f"{'tile':<28} {'shape':<44} {'calls':>5} {'ms':>7} " + " ".join(f"{s:>13}" for s in SECTIONS)
          + f" {'blocks':>7} {'conc':>5}")
    for (tile, shape), v in rows:
        secs = " ".join(f"{x / 1000:7.3f} {100 * x / max(v['wall'], 1e-9):4.0f}%" for x in v["sec"])
        print(f"{tile:<28} {shape:<44} {v['calls']:>5} {v['wall'] / 1000:7.3f} {secs} "
              f"{v['blocks'] // v['calls']:>7} {v['blk_wall'] / max(v['wall'], 1e-9):5.1f}")
    agg = [sum(v["sec"][k] for _, v in rows) for k in range(4)]
    print("# all dgrads: " + ", ".join(f"{s} {x / 1000:.3f} ms ({100 * x / max(total, 1e-9):.0f}%)"
                                       for s, x in zip(SECTIONS, agg)))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--warmup", type=int, default=4)
    ap.add_argument("--step_mode", default="one_stream", choices=["one_stream", "two_stream"])
    ap.add_argument("--dtype", default="bf16", choices=["bf16", "fp8"])
    ap.add_argument("--cap", type=int, default=1 << 20)
    a = ap.parse_args()
    recs = run(a)
    analyse(recs, f"ResNet-50 bs{a.batch} {a.dtype} {a.step_mode}")


if __name__ == "__main__":
    main()
