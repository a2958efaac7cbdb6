"""Cost of a cross-stream fork point on the main stream, by event kind (one MI355X):
two memory-bound kernels per iteration on the main stream, with a fork (event record on
main + wait on the side stream, which runs a tiny kernel) between them, for torch.cuda.Event
and the native StreamEvents ring in its three fence modes (csrc/runtime/events.cpp).  Then an
exactness check of the same-device hand-offs each mode would carry in the step: main writes
-> fork -> side reads, and side writes -> join -> main reads, on buffers large enough to be
spread over every XCD's L2.

    python bench/event_fence.py [--iters 400]
"""
import argparse
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=400)
    ap.add_argument("--mb", type=int, default=64)
    a = ap.parse_args()
    from pytorch_multiprocessing_distributed_amd.ops.native import C
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    main_s = torch.cuda.current_stream()
    side = torch.cuda.Stream()
    n = a.mb * (1 << 20) // 2
    x = torch.ones(n, dtype=torch.bfloat16, device=dev)
    small = torch.zeros(64, device=dev)
    rings = {m: C.StreamEvents(256, m, 0) for m in (0, 1, 2)}
    hm, hs = main_s.cuda_stream, side.cuda_stream

    def fork(kind):
        if kind == "none":
            return
        if kind == "torch":
            side.wait_stream(main_s)
        else:
            rings[int(kind[-1])].fork(hm, hs)

    def run(kind, iters):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(iters):
            x.mul_(1.0)
            fork(kind)
            if kind != "none":
                with torch.cuda.stream(side):
                    small.add_(1.0)
            x.mul_(1.0)
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) / iters * 1e6

    kinds = ["none", "torch", "mode0", "mode1", "mode2"]
    for k in kinds:
        run(k, 20)
    res = {k: [] for k in kinds}
    for _ in range(3):
        for k in kinds:
            res[k].append(round(run(k, a.iters), 2))
    base = min(res["none"])
    for k in kinds:
        print(json.dumps({"kind": k, "us_per_iter": res[k], "fork_cost_us": round(min(res[k]) - base, 2)}),
              flush=True)

    # exactness of the hand-offs (main -> side and side -> main) per mode
    idx = torch.arange(0, n, n // 4096 + 1, device=dev)
    for k in ["mode0", "mode1", "mode2"]:
        ring = rings[int(k[-1])]
        bufs = [torch.zeros(n, dtype=torch.float32, device=dev) for _ in range(2)]
        back = [torch.zeros(n, dtype=torch.float32, device=dev) for _ in range(2)]
        got_side = torch.zeros(a.iters, device=dev)
        got_main = torch.zeros(a.iters, device=dev)
        bad = 0
        for i in range(a.iters):
            b, r = bufs[i % 2], back[i % 2]
            b.fill_(float(i))                       # main writes
            ring.fork(hm, hs)
            with torch.cuda.stream(side):
                got_side[i] = b[idx].min() + b[idx].max() - float(i)   # side reads: == i
                r.fill_(float(i) + 0.5)             # side writes
            ring.fork(hs, hm)                       # join
            got_main[i] = r[idx].min() + r[idx].max() - float(i) - 1.0  # main reads: == i
        torch.cuda.synchronize()
        want = torch.arange(a.iters, device=dev, dtype=torch.float32)
        bad = int((got_side != want).sum()) + int((got_main != want).sum())
        print(json.dumps({"kind": k, "handoff_mismatches": bad, "checks": 2 * a.iters}), flush=True)
        assert bad == 0, f"{k}: {bad} stale reads"


if __name__ == "__main__":
    main()
