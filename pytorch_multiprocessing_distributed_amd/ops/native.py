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
    try:
        return importlib.import_module("pytorch_multiprocessing_distributed_amd._C")
    except ImportError:
        _ensure_built()
        return importlib.import_module("pytorch_multiprocessing_distributed_amd._C")


C = _load()


def available() -> bool:
    return C is not None
