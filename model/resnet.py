"""``model.resnet`` compatibility module (reference model/resnet.py API).

``ResNet18/34/50/101/152()`` return this framework's fused ResNet with the
reference's block counts, CIFAR stem, 10 classes and state_dict keys.  They
accept the reference's NCHW input (``net(torch.randn(1, 3, 32, 32))``); pass
``stem='imagenet', num_classes=1000`` for 224x224 training.
"""
from pytorch_multiprocessing_distributed_amd.models.resnet import (BasicBlock, Bottleneck,  # noqa: F401
                                                                   ResNet)
from pytorch_multiprocessing_distributed_amd.models import resnet as _r


def _mk(factory):
    def make(num_classes=10, stem="cifar", nchw_input=True):
        m = factory(num_classes=num_classes, stem=stem)
        m.nchw_input = nchw_input
        return m
    make.__doc__ = factory.__doc__
    return make


ResNet18 = _mk(_r.ResNet18)
ResNet34 = _mk(_r.ResNet34)
ResNet50 = _mk(_r.ResNet50)
ResNet101 = _mk(_r.ResNet101)
ResNet152 = _mk(_r.ResNet152)
