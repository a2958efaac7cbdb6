from .logger import AverageMeter, DeviceMeter, Logger, accuracy

__all__ = ["AverageMeter", "DeviceMeter", "Logger", "accuracy"]
