"""Reference-format observability helpers (utils.py:3-77 of the reference).

* :class:`AverageMeter` -- running val/sum/count/avg (utils.py:3-17).
* :class:`DeviceMeter` -- the same, but values may stay on the GPU until
  read, so the hot loop does not force a device->host sync every step
  (the reference does two ``.item()`` per step, main.py:113-114).
* :class:`Logger` -- space-separated text log, ints ``%04d``, floats
  ``%.6f``, append mode, fixed column count (utils.py:19-62); uses
  ``collections.abc`` (fixes SURVEY B7).
* :func:`accuracy` -- top-k precision, returns ``(res[0], correct.squeeze())``
  (utils.py:64-77).
"""
from __future__ import annotations

from collections.abc import Iterable

import torch


class AverageMeter:
    def __init__(self):
        self.reset()

    def reset(self):
        self.val = 0
        self.avg = 0
        self.sum = 0
        self.count = 0

    def update(self, val, n=1):
        self.val = val
        self.sum += val * n
        self.count += n
        self.avg = self.sum / self.count


class DeviceMeter:
    """AverageMeter whose updates may be 0-d device tensors (read lazily)."""

    def __init__(self):
        self.reset()

    def reset(self):
        self._val = 0.0
        self._sum = 0.0
        self.count = 0

    def update(self, val, n=1):
        self._val = val
        self._sum = self._sum + (val.detach().float() * n if torch.is_tensor(val) else val * n)
        self.count += n

    @staticmethod
    def _f(v):
        return float(v.item()) if torch.is_tensor(v) else float(v)

    @property
    def val(self):
        return self._f(self._val)

    @property
    def sum(self):
        return self._f(self._sum)

    @property
    def avg(self):
        return self.sum / self.count if self.count else 0.0


class Logger:
    def __init__(self, path, int_form=":04d", float_form=":.6f"):
        self.path = path
        self.int_form = int_form
        self.float_form = float_form
        self.width = 0

    def __len__(self):
        try:
            return len(self.read())
        except OSError:
            return 0

    def write(self, values):
        if not isinstance(values, Iterable) or isinstance(values, str):
            values = [values]
        if self.width == 0:
            self.width = len(values)
        assert self.width == len(values), "Inconsistent number of items."
        parts = []
        for v in values:
            if isinstance(v, bool):
                raise TypeError("Not supported type.")
            if isinstance(v, int):
                parts.append(("{" + self.int_form + "}").format(v))
            elif isinstance(v, float):
                parts.append(("{" + self.float_form + "}").format(v))
            elif isinstance(v, str):
                parts.append(v)
            else:
                raise TypeError("Not supported type.")
        with open(self.path, "a") as f:
            f.write(" ".join(parts) + "\n")

    def read(self):
        log = []
        with open(self.path, "r") as f:
            for line in f:
                values = []
                for v in line.split(" "):
                    try:
                        v = float(v)
                    except ValueError:
                        pass
                    values.append(v)
                log.append(values)
        return log


def accuracy(output, target, topk=(1,)):
    """Precision@k (percent) for the given k; returns (prec@topk[0], correct)."""
    maxk = max(topk)
    batch_size = target.size(0)
    _, pred = output.topk(maxk, 1, True, True)
    pred = pred.t()
    correct = pred.eq(target.view(1, -1).expand_as(pred))
    res = []
    for k in topk:
        correct_k = correct[:k].reshape(-1).float().sum(0)
        res.append(correct_k.mul_(100.0 / batch_size))
    return res[0], correct.squeeze()
