"""Loader for the in-tree gfx950 extension ``_C``.

The extension is built by ``csrc/build.py`` (or ``__graft_entry__.build()``)
into this package directory so the ``.so`` travels with the repository.  Build
provenance is content-based: ``_C.stamp.json`` records the sha256 of every
source the library was built from, and on import that hash is compared with
the sources in the tree.  A stale or unstamped library is rebuilt (printing
progress), or -- with ``PMD_NO_AUTOBUILD=1`` -- refused with an ImportError:
old kernels never run silently.  A missing or broken build raises loudly -- GPU
code paths never fall back to PyTorch silently.

Build VARIANTS are refused too: the stamp also records the compile flags, and a
library built with extra macros (``PMD_EXTRA_CFLAGS``, e.g. the timing-only
``-DPMD_TIMING_NO_ATOMICS`` that zeroes every BN statistic) or a non-default
optimisation level is rebuilt with the production flags -- or, with
``PMD_NO_AUTOBUILD=1``, refused -- unless ``PMD_ALLOW_VARIANT=1`` says the
variant is wanted (A/B scripts, ``bench/ab_so.sh``).  ``stamp_info()`` is what
``bench.py`` records in its JSON line (library digest, flags).
"""
from __future__ import annotations

import importlib
import os
import sys

_ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def _build_module():
    sys.path.insert(0, os.path.join(_ROOT, "csrc"))
    try:
        import build as _b  # csrc/build.py
    finally:
        sys.path.pop(0)
    return _b


PRODUCTION_OPT = ["-O3"]


def variant_reason(st) -> str:
    """Why the stamped library is not the production build ('' when it is)."""
    if st is None:
        return ""
    extra = str(st.get("extra_cflags", "")).strip()
    if extra:
        return f"built with extra flags {extra!r}"
    if st.get("opt", PRODUCTION_OPT) != PRODUCTION_OPT:
        return f"built with {st.get('opt')} instead of {PRODUCTION_OPT}"
    return ""


def _ensure_built():
    """Rebuild unless the library's stamp matches the sources in the tree AND records the
    production flags (or the variant is explicitly allowed)."""
    _b = _build_module()
    allow_variant = os.environ.get("PMD_ALLOW_VARIANT") == "1"
    if not allow_variant and os.environ.get("PMD_EXTRA_CFLAGS", "").strip():
        raise ImportError("PMD_EXTRA_CFLAGS is set: a variant build of the extension needs "
                          "PMD_ALLOW_VARIANT=1 (variants are A/B or timing-only builds)")
    st = _b.read_stamp()
    variant = "" if allow_variant else variant_reason(st)
    fresh = (os.path.exists(_b.target_path()) and st is not None
             and st.get("sources") == _b.source_digest() and not variant)
    if fresh:
        return
    if os.environ.get("PMD_NO_AUTOBUILD") == "1":
        why = ("no build stamp" if st is None else
               f"variant library: {variant} (set PMD_ALLOW_VARIANT=1 to use it)" if variant else
               "sources changed since the build")
        raise ImportError(f"refusing gfx950 extension {_b.target_path()} ({why}); "
                          "run `python csrc/build.py` (PMD_NO_AUTOBUILD=1 forbids rebuilding here)")
    if variant:
        print(f"[pmd] rebuilding the extension with the production flags ({variant})", flush=True)
    _b.build(verbose=True, force=bool(variant))


def stamp_info() -> dict:
    """Provenance of the loaded library for benchmark records."""
    _b = _build_module()
    st = _b.read_stamp() or {}
    if os.environ.get("PMD_EXT_DIR"):
        return {"lib_digest": None, "extra_cflags": None, "opt": None, "ext_dir": os.environ["PMD_EXT_DIR"]}
    return {"lib_digest": (st.get("library") or "")[:16] or None,
            "extra_cflags": st.get("extra_cflags", ""), "opt": " ".join(st.get("opt", []))}


def _load():
    import torch  # noqa: F401  (libtorch must be loaded first)
    ext_dir = os.environ.get("PMD_EXT_DIR")
    if ext_dir:   # an alternative build of _C (e.g. the host-ASan one, csrc/build.py --asan)
        import importlib.util as _ilu
        import sysconfig
        path = os.path.join(ext_dir, "_C" + sysconfig.get_config_var("EXT_SUFFIX"))
        spec = _ilu.spec_from_file_location("pytorch_multiprocessing_distributed_amd._C", path)
        if spec is None or not os.path.exists(path):
            raise ImportError(f"PMD_EXT_DIR={ext_dir}: no extension at {path}")
        mod = _ilu.module_from_spec(spec)
        sys.modules[spec.name] = mod
        spec.loader.exec_module(mod)
        return mod
    _ensure_built()
    return importlib.import_module("pytorch_multiprocessing_distributed_amd._C")


C = _load()
if os.environ.get("PMD_DET_STATS", "0") == "1":   # deterministic statistics (ops/functional.py)
    C.det_stats_set(True)


def available() -> bool:
    return C is not None
