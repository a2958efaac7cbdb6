"""MI355X-native multiprocess data-parallel ResNet training framework.

Capabilities mirror MOONJOOYOUNG/pytorch_multiprocessing-distributed
(one process per GPU via torch.multiprocessing.spawn, DistributedSampler
sharding, SyncBN, bucketed gradient all-reduce, SGD-nesterov + MultiStepLR,
rank-0 logs/plots, ``module.``-prefixed checkpoints), re-designed for gfx950:
hand-written HIP/MFMA kernels for the hot ops and RCCL over xGMI.
"""
__version__ = "0.1.0"
