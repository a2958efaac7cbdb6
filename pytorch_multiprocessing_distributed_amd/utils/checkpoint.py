"""Checkpoints.

* :func:`save_model` writes the reference's final checkpoint
  ``<save_path>/model_<epoch>.pth`` (main.py:74-77):
  ``torch.save`` zip container, an ``OrderedDict`` with ``_metadata``,
  ``module.``-prefixed keys from the data-parallel wrapper, fp32 tensors
  (int64 ``num_batches_tracked``), one storage per tensor, default (NCHW)
  contiguity -- so it loads with ``strict=True`` into the reference's
  ``ResNetXX()`` after stripping ``module.``.  Our parameters live as views
  of one flat arena with channels-last conv weights; each entry is copied
  out to its own dense storage before saving.
* :func:`save_resume` / :func:`load_resume` are a new capability (the
  reference has no resume): model + fused-SGD momentum + scheduler + epoch +
  sampler epoch + RNG states.
"""
from __future__ import annotations

import collections
import os
import random

import numpy as np
import torch


def export_state_dict(model):
    sd = model.state_dict()
    out = collections.OrderedDict()
    for k, v in sd.items():
        out[k] = v.detach().contiguous().clone()
    meta = getattr(sd, "_metadata", None)
    if meta is not None:
        out._metadata = meta
    return out


def save_model(model, save_path, epoch):
    path = os.path.join(save_path, "{0}_{1}.pth".format("model", epoch))
    torch.save(export_state_dict(model), path)
    return path


def load_model(model, path, strict=True, map_location="cpu"):
    """Load a reference-format checkpoint into ``model`` (wrapped or not)."""
    sd = torch.load(path, map_location=map_location, weights_only=True)
    has_prefix = next(iter(sd)).startswith("module.")
    wants_prefix = next(iter(model.state_dict())).startswith("module.")
    if has_prefix and not wants_prefix:
        sd = collections.OrderedDict((k[len("module."):], v) for k, v in sd.items())
    elif wants_prefix and not has_prefix:
        sd = collections.OrderedDict(("module." + k, v) for k, v in sd.items())
    with torch.no_grad():
        own = model.state_dict()
        missing = [k for k in own if k not in sd]
        unexpected = [k for k in sd if k not in own]
        if strict and (missing or unexpected):
            raise RuntimeError(f"checkpoint mismatch: missing={missing} unexpected={unexpected}")
        for k, v in sd.items():
            if k in own:
                own[k].copy_(v)       # in place: keeps the flat-arena views intact
    return model


def save_resume(path, model, optimizer, scheduler, epoch, sampler_epoch=None):
    state = {
        "model": export_state_dict(model),
        "optimizer": optimizer.state_dict() if optimizer is not None else None,
        "scheduler": scheduler.state_dict() if scheduler is not None else None,
        "epoch": epoch,
        "sampler_epoch": sampler_epoch if sampler_epoch is not None else epoch,
        "rng": {
            "torch": torch.get_rng_state(),
            "cuda": torch.cuda.get_rng_state_all() if torch.cuda.is_available() else [],
            "numpy": torch.from_numpy(np.frombuffer(
                np.random.get_state()[1].tobytes(), dtype=np.uint8).copy()),
            "python": torch.tensor(list(random.getstate()[1]), dtype=torch.int64),
        },
    }
    tmp = path + ".tmp"
    torch.save(state, tmp)
    os.replace(tmp, path)
    return path


def load_resume(path, model, optimizer=None, scheduler=None, map_location="cpu"):
    state = torch.load(path, map_location=map_location, weights_only=True)
    load_model_state(model, state["model"])
    if optimizer is not None and state.get("optimizer") is not None:
        optimizer.load_state_dict(state["optimizer"])
    if scheduler is not None and state.get("scheduler") is not None:
        scheduler.load_state_dict(state["scheduler"])
    rng = state.get("rng", {})
    if "torch" in rng:
        torch.set_rng_state(rng["torch"])
    if rng.get("cuda") and torch.cuda.is_available():
        torch.cuda.set_rng_state_all(rng["cuda"])
    return state["epoch"], state.get("sampler_epoch", state["epoch"])


def load_model_state(model, sd):
    with torch.no_grad():
        own = model.state_dict()
        for k, v in sd.items():
            own[k].copy_(v)
