"""Loader for the in-tree gfx950 extension ``_C``.

The extension is built by ``csrc/build.py`` (or ``__graft_entry__.build()``)
into this package directory so the ``.so`` travels with the repository.  On
import we rebuild only if a source is newer than the library (cheap mtime
check) and then load it; a missing or broken build raises loudly -- GPU code
paths never fall back to PyTorch silently.
"""
from __future__ import annotations

import importlib
import os
import sys

_ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def _ensure_built():
    sys.path.insert(0, os.path.join(_ROOT, "csrc"))
    try:
        import build as _b  # csrc/build.py
    finally:
        sys.path.pop(0)
    if os.environ.get("PMD_NO_AUTOBUILD") == "1" and os.path.exists(_b.target_path()):
        return
    _b.build(verbose=False)


def _load():
    import torch  # noqa: F401  (libtorch must be loaded first)
    try:
        return importlib.import_module("pytorch_multiprocessing_distributed_amd._C")
    except ImportError:
        _ensure_built()
        return importlib.import_module("pytorch_multiprocessing_distributed_amd._C")


C = _load()


def available() -> bool:
    return C is not None
