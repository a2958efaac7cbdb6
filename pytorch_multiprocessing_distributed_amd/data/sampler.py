"""Per-rank sharding identical to ``torch.utils.data.DistributedSampler``
(reference data.py:31-37; torch:utils/data/distributed.py:102-134):

  shuffle : randperm(N, generator seeded with seed + epoch)
  pad     : wrap indices to ceil(N / W) * W (drop_last=False)
  shard   : indices[rank : total : W]

The reference never calls ``set_epoch``, so its shuffle is the
same every epoch; ``fixed_order=True`` reproduces that, the default advances
the epoch like a correct training script.
"""
from __future__ import annotations

import math

import torch


class DistributedSampler:
    def __init__(self, num_samples: int, num_replicas: int = 1, rank: int = 0,
                 shuffle: bool = True, seed: int = 0, drop_last: bool = False,
                 fixed_order: bool = False):
        if rank >= num_replicas or rank < 0:
            raise ValueError(f"invalid rank {rank} for {num_replicas} replicas")
        self.n = num_samples
        self.num_replicas = num_replicas
        self.rank = rank
        self.shuffle = shuffle
        self.seed = seed
        self.drop_last = drop_last
        self.fixed_order = fixed_order
        self.epoch = 0
        if drop_last and num_samples % num_replicas != 0:
            self.num_samples = math.ceil((num_samples - num_replicas) / num_replicas)
        else:
            self.num_samples = math.ceil(num_samples / num_replicas)
        self.total_size = self.num_samples * num_replicas

    def set_epoch(self, epoch: int):
        if not self.fixed_order:
            self.epoch = epoch

    def indices(self) -> list:
        if self.shuffle:
            g = torch.Generator()
            g.manual_seed(self.seed + self.epoch)
            idx = torch.randperm(self.n, generator=g).tolist()
        else:
            idx = list(range(self.n))
        if not self.drop_last:
            pad = self.total_size - len(idx)
            if pad <= len(idx):
                idx += idx[:pad]
            else:
                idx += (idx * math.ceil(pad / len(idx)))[:pad]
        else:
            idx = idx[: self.total_size]
        assert len(idx) == self.total_size
        out = idx[self.rank: self.total_size: self.num_replicas]
        assert len(out) == self.num_samples
        return out

    def __iter__(self):
        return iter(self.indices())

    def __len__(self):
        return self.num_samples
