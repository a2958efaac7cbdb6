"""Device-resident data loaders (replace DataLoader workers, reference data.py:39-53).

* :class:`DeviceLoader` keeps the whole uint8 dataset on the GPU (CIFAR-10 is
  150 MB; an MI355X has 288 GB) and produces each batch with one fused
  augmentation kernel (crop+pad / flip / normalise / NHWC / cast) from the
  DistributedSampler shard -- no worker processes, no pinned-memory thread,
  no per-step host->device copy.
* :class:`SyntheticImageNet` generates ImageNet-shaped NHWC bf16 batches on
  device (BASELINE north star: synthetic data, random-init weights).

Per-rank batch = int(global_batch / world_size), exactly like the reference
(data.py:39); ``len()`` follows DataLoader's drop_last=False rule.
"""
from __future__ import annotations

import math

import numpy as np
import torch

from .sampler import DistributedSampler

_M64 = (1 << 64) - 1


def _mix32_np(z):
    z = (z + np.uint64(0x9E3779B97F4A7C15)) & np.uint64(_M64)
    z = ((z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)) & np.uint64(_M64)
    z = ((z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)) & np.uint64(_M64)
    return ((z ^ (z >> np.uint64(31))) >> np.uint64(16)).astype(np.uint32)


def augment_params(sample_idx: np.ndarray, seed: int, epoch: int, pad: int = 8):
    """(oy, ox, flip) per sample -- the same counter hash as cifar_augment_kernel."""
    with np.errstate(over="ignore"):
        z = (np.uint64(seed) * np.uint64(1315423911) + np.uint64(epoch) * np.uint64(2654435761)
             + sample_idx.astype(np.uint64))
        h = _mix32_np(z).astype(np.int64)
    span = 2 * pad + 1
    return h % span, (h // span) % span, (h >> 24) & 1


def cifar_augment_torch(data, idx, cpad, train, pad, seed, epoch, dtype):
    """CPU reference of csrc/kernels/data.hip:cifar_augment_kernel."""
    imgs = data[idx].float() / 255.0                     # [B,32,32,3]
    b = imgs.shape[0]
    if train:
        oy, ox, flip = augment_params(idx.cpu().numpy(), seed, epoch, pad)
        padded = torch.zeros(b, 32 + 2 * pad, 32 + 2 * pad, 3)
        padded[:, pad:pad + 32, pad:pad + 32] = imgs
        out = torch.empty_like(imgs)
        for i in range(b):
            crop = padded[i, oy[i]:oy[i] + 32, ox[i]:ox[i] + 32]
            out[i] = crop.flip(1) if flip[i] else crop
        imgs = out
    x = (imgs - 0.5) / 0.5
    if cpad > 3:
        x = torch.nn.functional.pad(x, (0, cpad - 3))
    return x.to(dtype).contiguous()


class DeviceLoader:
    def __init__(self, images, labels, global_batch, world_size=1, rank=0, train=True,
                 device="cpu", dtype=torch.float32, cpad=3, seed=0, shuffle=True,
                 fixed_order=False, pad=8, max_batches=None):
        self.device = torch.device(device)
        self.images = images.to(self.device).contiguous()
        self.labels = labels.to(self.device).long()
        self.batch = int(global_batch / world_size)          # reference data.py:39
        if self.batch < 1:
            raise ValueError("global batch smaller than world size")
        self.sampler = DistributedSampler(len(images), world_size, rank, shuffle=shuffle,
                                          fixed_order=fixed_order)
        self.train = train
        self.dtype = dtype
        self.cpad = cpad
        self.seed = seed
        self.pad = pad
        self.epoch = 0
        self.max_batches = max_batches
        self.dataset_len = len(images)

    def set_epoch(self, epoch):
        self.epoch = epoch
        self.sampler.set_epoch(epoch)

    def __len__(self):
        n = math.ceil(len(self.sampler) / self.batch)
        return min(n, self.max_batches) if self.max_batches else n

    def __iter__(self):
        idx_all = torch.tensor(self.sampler.indices(), dtype=torch.int64, device=self.device)
        use_hip = self.device.type == "cuda"
        if use_hip:
            from ..ops.native import C
        for i in range(len(self)):
            idx = idx_all[i * self.batch: (i + 1) * self.batch]
            if use_hip:
                x = C.cifar_augment(self.images, idx, self.cpad, self.train, self.pad, self.seed,
                                    self.epoch, self.dtype == torch.bfloat16)
            else:
                x = cifar_augment_torch(self.images, idx, self.cpad, self.train, self.pad,
                                        self.seed, self.epoch, self.dtype)
            yield x, self.labels[idx]


class SyntheticImageNet:
    """Random-init-equivalent ImageNet batches, generated on device per step."""

    def __init__(self, batch, image=224, classes=1000, steps=100, device="cpu",
                 dtype=torch.float32, cpad=3, seed=0, dataset_len=1281167):
        self.batch = batch
        self.image = image
        self.classes = classes
        self.steps = steps
        self.device = torch.device(device)
        self.dtype = dtype
        self.cpad = cpad
        self.seed = seed
        self.epoch = 0
        self.dataset_len = dataset_len
        self._pf_stream = None
        self._pf_transform = None
        self._pf = {}

    def set_epoch(self, epoch):
        self.epoch = epoch
        self._pf.clear()

    def prefetch(self, stream, transform=None):
        """Generate every batch one step ahead on ``stream`` (the two-stream step's weight-gradient
        stream, idle during the forward): :meth:`next_batch` ``(i)`` hands out batch i -- made on
        ``stream`` while step i-1 ran, the current stream waiting for it -- and queues batch i+1.
        The same batches and the same per-step generation work, off the main stream's critical
        path (a prefetching data loader).  ``None``: generate in place.  ``transform``: applied to
        each batch's images on ``stream`` too (the model's input layout step,
        ops/functional.py s2d_input_prefetch); tensors it attaches as ``x._pmd_*`` attributes
        are handed to the consuming stream with the batch."""
        self._pf_stream = stream
        self._pf_transform = transform
        self._pf.clear()

    def _made_on_side(self, i):
        with torch.cuda.stream(self._pf_stream):
            x, y = self.batch_at(i)
            if self._pf_transform is not None:
                x = self._pf_transform(x)
            ev = torch.cuda.Event()
            ev.record(self._pf_stream)
        return x, y, ev

    def next_batch(self, i):
        if self._pf_stream is None or self.device.type != "cuda":
            return self.batch_at(i)
        cur = torch.cuda.current_stream(self.device)
        b = self._pf.pop(i, None)
        x, y, ev = b if b is not None else self._made_on_side(i)
        cur.wait_event(ev)
        x.record_stream(cur)            # allocated on the prefetch stream, consumed here
        y.record_stream(cur)
        xs = getattr(x, "_pmd_s2d_in", None)
        if xs is not None:
            xs.record_stream(cur)
        if i + 1 < self.steps:
            self._pf[i + 1] = self._made_on_side(i + 1)
        return x, y

    def __len__(self):
        return self.steps

    def batch_at(self, step):
        s = self.seed * 1000003 + self.epoch * 100003 + step
        if self.device.type == "cuda":
            from ..ops.native import C
            x, y = C.synth_images(self.batch, self.image, self.image, self.cpad, 3, self.classes, s,
                                  self.device.index or 0)
            return x, y
        g = torch.Generator().manual_seed(s)
        x = torch.randn(self.batch, self.image, self.image, 3, generator=g)
        if self.cpad > 3:
            x = torch.nn.functional.pad(x, (0, self.cpad - 3))
        y = torch.randint(0, self.classes, (self.batch,), generator=g)
        return x.to(self.dtype), y

    def __iter__(self):
        for i in range(self.steps):
            yield self.next_batch(i)
