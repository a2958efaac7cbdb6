import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) GPU")
    config.addinivalue_line("markers", "slow: multi-process or long-running test")


def pytest_collection_modifyitems(config, items):
    # the multi-process GPU tests run last: they take most of the GPU suite's time, and under -x
    # a failure there no longer hides the single-process kernel / model tests behind it (the CPU
    # suite keeps its file order)
    last = [it for it in items if "slow" in it.keywords and "gpu" in it.keywords]
    if last:
        items[:] = [it for it in items if not ("slow" in it.keywords and "gpu" in it.keywords)] + last
    import torch
    if torch.cuda.is_available():
        return
    skip = pytest.mark.skip(reason="no GPU in this container")
    for it in items:
        if "gpu" in it.keywords:
            it.add_marker(skip)
