from . import functional, torch_prims

__all__ = ["functional", "torch_prims"]
