from .resnet import (BasicBlock, BatchNorm, Bottleneck, Conv2d, MODELS, ResNet, ResNet18,
                     ResNet18Full, ResNet34, ResNet50, ResNet101, ResNet152, build_model)

__all__ = ["BasicBlock", "BatchNorm", "Bottleneck", "Conv2d", "MODELS", "ResNet", "ResNet18",
           "ResNet18Full", "ResNet34", "ResNet50", "ResNet101", "ResNet152", "build_model"]
