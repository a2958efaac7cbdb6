"""Per-dispatch sequence of ONE training step from a rocprofv3 (rocpd) kernel trace:
kernel (template args kept), grid, workgroup, VGPR/AGPR, LDS and duration, in issue order.
Used to map each conv/BN dispatch to its ResNet layer.

    python bench/prof_sequence.py gpurun_out/prof/run_results.db [--step -2] [--marker synth_images_kernel]
"""
import argparse
import re
import sqlite3


def short(name):
    name = re.sub(r"\(.*\)$", "", name)
    return name.replace("void ", "").replace("pmd::", "")[:64]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--step", type=int, default=-2, help="which marker-delimited step (python index)")
    ap.add_argument("--marker", default="synth_images_kernel")
    ap.add_argument("--min_us", type=float, default=0.0)
    a = ap.parse_args()
    c = sqlite3.connect(a.db)
    ks = c.execute("select name, start, end, grid_x, grid_y, grid_z, workgroup_x, vgpr_count, "
                   "accum_vgpr_count, lds_size from kernels order by start").fetchall()
    marks = [i for i, k in enumerate(ks) if a.marker in k[0]] + [len(ks)]
    s = a.step if a.step >= 0 else len(marks) - 1 + a.step
    seg = ks[marks[s]:marks[s + 1]]
    t0 = seg[0][1]
    tot = 0.0
    for n, st, en, gx, gy, gz, wx, vg, ag, lds in seg:
        d = (en - st) / 1e3
        tot += d
        if d < a.min_us:
            continue
        print(f"{(st - t0) / 1e3:9.1f} {d:8.1f}us  {short(n):64s} grid={gx // max(wx, 1)}x{gy}x{gz} "
              f"wg={wx} v={vg}/{ag} lds={lds}")
    print(f"# {len(seg)} dispatches, busy {tot / 1e3:.2f} ms, span {(seg[-1][2] - t0) / 1e6:.2f} ms")


if __name__ == "__main__":
    main()
