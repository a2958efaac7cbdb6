from .comm import Comm, get_comm
from .dp import DataParallel
from .flat import FlatParams, flatten_module

__all__ = ["Comm", "get_comm", "DataParallel", "FlatParams", "flatten_module"]
