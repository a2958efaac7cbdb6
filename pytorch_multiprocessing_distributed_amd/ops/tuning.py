"""Per-shape kernel tuning tables: the framework's ``cudnn.benchmark`` state
(reference main.py:45 sets ``torch.backends.cudnn.benchmark = True``).

The native conv (fwd/dgrad) and wgrad launchers time their candidate kernels
the first time they meet a shape (kernels/conv_igemm.hip ``tune``,
kernels/conv_wgrad.hip ``wgrad_tune``) and cache the winner.  This module makes
that cache

  * persistent -- :func:`save` / :func:`load` a JSON table (an offline-tuned
    table for a model/batch skips the host-synchronising timing runs of the
    first step entirely), and
  * rank-consistent -- :func:`sync` broadcasts rank 0's table and every rank
    adopts it, so all ranks run the same kernel for every shape (identical
    per-rank step time, no per-rank timing noise in the kernel choice).

  * deterministic by default -- :func:`load_default` installs the committed
    table for this device (``ops/tables/*.json``, produced offline by a
    majority vote over several independently autotuned processes,
    ``bench/make_tune_table.py``).  Step-0 timing of candidates on a live,
    two-stream step is noisy: two fresh processes on the same box disagreed
    on 4 of 68 shapes (``profiles/fresh_vs_warm_r03.txt``), so the run-to-run
    kernel mix -- and the headline number -- varied with it.  Shapes the table
    does not cover are still autotuned online.

Table format: ``{"version": 1, "device": <name>, "arch": <gcnArchName>,
"conv": [[13 key ints, choice], ...], "wgrad": [[11 key ints, variant], ...]}``;
keys are the launch shapes (N, H, W, C, P/OH, Q/OW, K, R, S, stride, pad[,
dgrad, stats]).
"""
from __future__ import annotations

import glob
import hashlib
import json
import os

import torch

CONV_KEY, WGRAD_KEY = 13, 11
TABLE_DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)), "tables")


def device_arch() -> str:
    if not torch.cuda.is_available():
        return "cpu"
    return torch.cuda.get_device_properties(torch.cuda.current_device()).gcnArchName.split(":")[0]


def _c():
    from .native import C
    return C


def export_table() -> dict:
    C = _c()
    conv = C.conv_autotune_export()
    wg = C.wgrad_autotune_export()
    dev = torch.cuda.get_device_name() if torch.cuda.is_available() else "cpu"
    return {"version": 1, "device": dev, "arch": device_arch(),
            "conv": [conv[i:i + CONV_KEY + 1] for i in range(0, len(conv), CONV_KEY + 1)],
            "wgrad": [wg[i:i + WGRAD_KEY + 1] for i in range(0, len(wg), WGRAD_KEY + 1)]}


def import_table(tab: dict) -> int:
    """Merge a table into the live tuner caches; returns the number of entries."""
    if tab.get("version") != 1:
        raise ValueError(f"unknown tuning table version {tab.get('version')!r}")
    C = _c()
    n = 0
    conv = [v for e in tab.get("conv", []) for v in e]
    wg = [v for e in tab.get("wgrad", []) for v in e]
    if conv:
        n += C.conv_autotune_import([int(v) for v in conv])
    if wg:
        n += C.wgrad_autotune_import([int(v) for v in wg])
    return n


def save(path: str) -> dict:
    tab = export_table()
    d = os.path.dirname(os.path.abspath(path))
    os.makedirs(d, exist_ok=True)
    with open(path, "w") as f:
        json.dump(tab, f)
    return tab


def load(path: str) -> int:
    with open(path) as f:
        return import_table(json.load(f))


def sync(group=None) -> int:
    """Collective: every rank adopts rank 0's tuning table (call after the first
    step, when every shape has been met).  Returns the entries adopted."""
    import torch.distributed as dist
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size(group) == 1:
        return 0
    obj = [export_table() if dist.get_rank(group) == 0 else None]
    dist.broadcast_object_list(obj, src=0, group=group)
    C = _c()
    C.conv_autotune_clear()
    C.wgrad_autotune_clear()
    return import_table(obj[0])


def table_hash(tab: dict | None = None) -> str:
    """Short digest of the kernel choices (live caches by default): two runs
    with the same hash ran the same kernel for every tuned shape."""
    tab = export_table() if tab is None else tab
    key = json.dumps({"conv": sorted(tab.get("conv", [])), "wgrad": sorted(tab.get("wgrad", []))})
    return hashlib.sha1(key.encode()).hexdigest()[:12]


def default_tables(arch: str | None = None):
    """Committed tables whose ``arch`` matches this device (gfx950)."""
    arch = device_arch() if arch is None else arch
    out = []
    for path in sorted(glob.glob(os.path.join(TABLE_DIR, "*.json"))):
        try:
            with open(path) as f:
                tab = json.load(f)
        except (OSError, ValueError):
            continue
        if tab.get("version") == 1 and tab.get("arch", "gfx950") == arch:
            out.append((path, tab))
    return out


def load_default() -> tuple[str, int]:
    """Install every committed table for this device.  Entries are keyed by the
    exact launch shape (batch included), so a table for another model or
    batch size simply never matches; those shapes are autotuned online.
    Returns (source label, entries installed)."""
    if os.environ.get("PMD_TUNE_TABLE", "1") == "0":
        return "online", 0
    n, names = 0, []
    for path, tab in default_tables():
        n += import_table(tab)
        names.append(os.path.basename(path))
    return ("table:" + "+".join(names) if names else "online"), n
