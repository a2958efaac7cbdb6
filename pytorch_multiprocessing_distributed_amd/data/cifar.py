"""CIFAR-10 readers (no torchvision in this image) and a synthetic stand-in.

The reference reads ``./cifar10_data`` through ``torchvision.datasets.CIFAR10``
(data.py:21-28), i.e. the ``cifar-10-batches-py`` pickles.  We read:
  * ``cifar-10-batches-bin`` (raw records: 1 label byte + 3072 CHW bytes), or
  * ``cifar-10-batches-py`` through a *restricted* unpickler that can only
    rebuild numpy arrays / dicts / lists (nothing executable), or
  * a deterministic synthetic CIFAR-shaped set (50000/10000, uint8) when no
    data is present -- this container has no network and ships no dataset.

All return uint8 ``[N, 32, 32, 3]`` (HWC) images and int64 labels, the layout
the on-device augmentation kernel consumes.
"""
from __future__ import annotations

import io
import os
import pickle

import numpy as np
import torch

TRAIN_LEN, TEST_LEN = 50000, 10000


class _SafeUnpickler(pickle.Unpickler):
    _ALLOWED = {
        ("numpy.core.multiarray", "_reconstruct"), ("numpy._core.multiarray", "_reconstruct"),
        ("numpy", "ndarray"), ("numpy", "dtype"), ("numpy.core.multiarray", "scalar"),
        ("numpy._core.multiarray", "scalar"), ("builtins", "list"), ("builtins", "dict"),
    }

    def find_class(self, module, name):
        if (module, name) in self._ALLOWED:
            return super().find_class(module, name)
        raise pickle.UnpicklingError(f"refusing to load {module}.{name} from a CIFAR batch")


def _load_py_batch(path):
    with open(path, "rb") as f:
        d = _SafeUnpickler(io.BytesIO(f.read()), encoding="latin1").load()
    data = np.asarray(d["data"], dtype=np.uint8).reshape(-1, 3, 32, 32).transpose(0, 2, 3, 1)
    labels = np.asarray(d.get("labels", d.get("fine_labels")), dtype=np.int64)
    return data, labels


def _load_bin_batch(path):
    raw = np.fromfile(path, dtype=np.uint8).reshape(-1, 3073)
    labels = raw[:, 0].astype(np.int64)
    data = raw[:, 1:].reshape(-1, 3, 32, 32).transpose(0, 2, 3, 1)
    return np.ascontiguousarray(data), labels


def load_cifar10(root: str, train: bool):
    """Returns (uint8 [N,32,32,3], int64 [N]) or None if no data under root."""
    py = os.path.join(root, "cifar-10-batches-py")
    bn = os.path.join(root, "cifar-10-batches-bin")
    if os.path.isdir(py):
        names = [f"data_batch_{i}" for i in range(1, 6)] if train else ["test_batch"]
        parts = [_load_py_batch(os.path.join(py, n)) for n in names]
    elif os.path.isdir(bn):
        names = [f"data_batch_{i}.bin" for i in range(1, 6)] if train else ["test_batch.bin"]
        parts = [_load_bin_batch(os.path.join(bn, n)) for n in names]
    else:
        return None
    data = np.concatenate([p[0] for p in parts])
    labels = np.concatenate([p[1] for p in parts])
    return torch.from_numpy(np.ascontiguousarray(data)), torch.from_numpy(labels)


def synthetic_cifar10(train: bool, n: int | None = None, seed: int = 0, classes: int = 10):
    """Deterministic CIFAR-shaped uint8 data with a weak class signal (a
    per-class colour bias) so training curves move."""
    n = n if n is not None else (TRAIN_LEN if train else TEST_LEN)
    g = torch.Generator().manual_seed(seed + (0 if train else 1))
    labels = torch.randint(0, classes, (n,), generator=g)
    base = torch.randint(0, 256, (n, 32, 32, 3), generator=g, dtype=torch.int32)
    bias = (torch.arange(classes).view(-1, 1) * torch.tensor([37, 91, 53]).view(1, 3)) % 96 - 48
    img = (base // 2 + 64 + bias[labels].view(n, 1, 1, 3)).clamp(0, 255).to(torch.uint8)
    return img, labels


def get_cifar10(root: str, train: bool, synthetic: bool = False, n: int | None = None):
    if not synthetic:
        got = load_cifar10(root, train)
        if got is not None:
            if n is not None:
                got = (got[0][:n], got[1][:n])
            return got
    return synthetic_cifar10(train, n=n)
