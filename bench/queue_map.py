"""Which hardware queue carried which HIP stream's kernels (rocprofv3 rocpd trace).

The xGMI SyncBN exchange spins inside a kernel waiting for its peers; if two HIP streams
that both carry cross-rank waits (the exchange, an RCCL collective) shared one hardware
queue, a rank could park the collective behind its own spinning exchange (docs/
ARCHITECTURE.md, "Streams -> hardware queues").  This tabulates, per process (rank):
stream -> queue ids and the kernel families each stream ran, and flags any queue that
carries more than one stream.

    python bench/queue_map.py gpurun_out/<dir>/run_results.db [--skip-kernels N]
"""
import argparse
import collections
import re
import sqlite3


def family(name):
    n = re.sub(r"\(.*\)$", "", name).replace("void ", "").replace("pmd::", "")
    n = re.sub(r"<.*", "", n)
    if "nccl" in n.lower() or "rccl" in n.lower() or n.startswith("__amd_rocclr"):
        return n[:40]
    return n[:40]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--steps-only", action="store_true",
                    help="only kernels inside the training steps (first to last synth_images_kernel "
                         "of each process): setup-time copies / fills on library streams excluded")
    a = ap.parse_args()
    c = sqlite3.connect(a.db)
    rows = c.execute("select pid, stream_id, stream, queue_id, queue, name, start from kernels").fetchall()
    if a.steps_only:
        win = {}
        for pid, _sid, _sn, _qid, _qn, name, t in rows:
            if "synth_images_kernel" in name:
                lo, hi = win.get(pid, (t, t))
                win[pid] = (min(lo, t), max(hi, t))
        rows = [r for r in rows if r[0] in win and win[r[0]][0] <= r[6] <= win[r[0]][1]]
    rows = [r[:6] for r in rows]
    per = collections.defaultdict(lambda: collections.defaultdict(lambda: {"queues": collections.Counter(),
                                                                          "fams": collections.Counter()}))
    for pid, sid, sname, qid, qname, name in rows:
        e = per[pid][(sid, sname)]
        e["queues"][(qid, qname)] += 1
        e["fams"][family(name)] += 1
    bad = 0
    for pid in sorted(per):
        print(f"== process {pid}: {len(per[pid])} stream(s)")
        q2s = collections.defaultdict(set)
        for (sid, sname), e in sorted(per[pid].items()):
            qs = ", ".join(f"{qn or qid} x{n}" for (qid, qn), n in e["queues"].most_common())
            fams = ", ".join(f"{f} x{n}" for f, n in e["fams"].most_common(6))
            print(f"  stream {sid} ({sname}): queues [{qs}]\n      kernels: {fams}")
            for (qid, qn) in e["queues"]:
                q2s[qn or qid].add((sid, sname))
        for q, ss in sorted(q2s.items(), key=lambda kv: str(kv[0])):
            if len(ss) > 1:
                bad += 1
                names = ", ".join(f"{sid} ({sn})" for sid, sn in sorted(ss))
                print(f"  !! {q} carries streams {names}")
    print("one queue per stream" if bad == 0 else f"{bad} shared queue(s)")


if __name__ == "__main__":
    main()
