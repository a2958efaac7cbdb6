"""Loader for the in-tree gfx950 extension ``_C``.

The extension is built by ``csrc/build.py`` (or ``__graft_entry__.build()``)
into this package directory so the ``.so`` travels with the repository.  Build
provenance is content-based: ``_C.stamp.json`` records the sha256 of every
source the library was built from, and on import that hash is compared with
the sources in the tree.  A stale or unstamped library is rebuilt (printing
progress), or -- with ``PMD_NO_AUTOBUILD=1`` -- refused with an ImportError:
old kernels never run silently.  A missing or broken build raises loudly -- GPU
code paths never fall back to PyTorch silently.
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


def _ensure_built():
    """Rebuild unless the library's stamp matches the sources in the tree."""
    _b = _build_module()
    st = _b.read_stamp()
    fresh = (os.path.exists(_b.target_path()) and st is not None
             and st.get("sources") == _b.source_digest())
    if fresh:
        return
    if os.environ.get("PMD_NO_AUTOBUILD") == "1":
        why = "no build stamp" if st is None else "sources changed since the build"
        raise ImportError(f"stale gfx950 extension {_b.target_path()} ({why}); "
                          "run `python csrc/build.py` (PMD_NO_AUTOBUILD=1 forbids rebuilding here)")
    _b.build(verbose=True)


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


def available() -> bool:
    return C is not None
