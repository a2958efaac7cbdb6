"""``utils`` compatibility module (reference utils.py API): AverageMeter,
Logger (same text format), accuracy."""
from pytorch_multiprocessing_distributed_amd.utils.logger import (AverageMeter, DeviceMeter,  # noqa: F401
                                                                  Logger, accuracy)
