"""``data`` compatibility module: ``get_loader(args, rank, world_size)``
returns (train_loader, test_loader) like the reference, backed by the
device-resident CIFAR-10 loaders (DistributedSampler sharding, per-rank batch
``int(args.batch_size / args.world_size)``).  ``args`` needs ``batch_size``
and ``world_size``; ``data_root``/``synthetic``/``train_samples`` are optional.
"""
import torch

from pytorch_multiprocessing_distributed_amd.engine.train import build_loaders


def get_loader(args, rank, world_size):
    for k, v in (("stem", "cifar"), ("data_root", "./cifar10_data"), ("synthetic", False),
                 ("train_samples", None), ("max_steps", None), ("eval_batches", None),
                 ("fixed_order", False), ("image_size", 32), ("num_classes", 10),
                 ("steps_per_epoch", 100)):
        if not hasattr(args, k):
            setattr(args, k, v)
    on_gpu = torch.cuda.is_available()
    dev = torch.device("cuda", torch.cuda.current_device()) if on_gpu else torch.device("cpu")
    dtype = torch.bfloat16 if on_gpu else torch.float32
    return build_loaders(args, rank, args.world_size, dev, dtype, 8 if on_gpu else 3)
