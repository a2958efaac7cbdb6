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
    a = ap.parse_args()
    c = sqlite3.connect(a.db)
    rows = c.execute("select pid, stream_id, stream, queue_id, queue, name from kernels").fetchall()
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
            for (qid, _qn) in e["queues"]:
                q2s[qid].add(sid)
        for qid, ss in sorted(q2s.items()):
            if len(ss) > 1:
                bad += 1
                print(f"  !! queue {qid} carries streams {sorted(ss)}")
    print("one queue per stream" if bad == 0 else f"{bad} shared queue(s)")


if __name__ == "__main__":
    main()
