"""Checkpoint I/O in the reference's format, and its model factory.

* :func:`save_checkpoint` writes what train.py:151-161 writes every ``save_step``:
  ``torch.save({"model": <240-key state_dict>, "optimizer": <Adam state_dict>}, "<step>.pth.tar")``
  (the reference saves ``model.module.state_dict()`` of its DataParallel wrapper: the bare
  model's keys, as here).
* :func:`get_model` is utils/model.py:11-34: build ``FastSpeech2``, restore
  ``<ckpt_path>/<restore_step>.pth.tar`` when ``args.restore_step`` is set, and in training also a
  :class:`ScheduledOptim` whose Noam step counter starts at ``restore_step`` (model/optimizer.py:19)
  with the saved Adam moments restored. Loading uses ``torch.load(..., weights_only=True)``: the
  checkpoint holds only tensors and plain containers, so nothing in the file is executed (the
  reference's ``weights_only=False`` would unpickle arbitrary objects).
"""
import os

import torch

from .model import FastSpeech2
from .optimizer import ScheduledOptim


def checkpoint_path(train_config, step):
    return os.path.join(train_config["path"]["ckpt_path"], "{}.pth.tar".format(step))


def save_checkpoint(path, model, optimizer):
    """train.py:151-161. ``model`` may be a DDP / DataParallel wrapper (its ``.module`` is saved)."""
    core = model.module if hasattr(model, "module") else model
    os.makedirs(os.path.dirname(path) or ".", exist_ok=True)
    torch.save({"model": core.state_dict(), "optimizer": optimizer._optimizer.state_dict()}, path)


def _numpy_scalar_globals():
    """Reference checkpoints carry numpy float64 learning rates in the Adam param_groups
    (ScheduledOptim computes lr with numpy): allow only numpy's scalar / dtype reconstructors,
    which rebuild a number from its dtype and bytes and execute nothing else."""
    import numpy as np

    core = getattr(np, "_core", None) or np.core
    allowed = [core.multiarray.scalar, np.dtype]
    allowed += [type(np.dtype(t)) for t in ("float64", "float32", "int64")]
    return allowed


def load_checkpoint(path, map_location=None):
    with torch.serialization.safe_globals(_numpy_scalar_globals()):
        return torch.load(path, map_location=map_location, weights_only=True)


def get_model(args, configs, device, train=False):
    """utils/model.py:11-34: returns the model (eval) or (model, ScheduledOptim) (train)."""
    preprocess_config, model_config, train_config = configs
    model = FastSpeech2(preprocess_config, model_config).to(device)
    ckpt = None
    if args.restore_step:
        ckpt = load_checkpoint(checkpoint_path(train_config, args.restore_step), map_location=device)
        model.load_state_dict(ckpt["model"])
    if train:
        optim = ScheduledOptim(model, train_config, model_config, args.restore_step)
        if args.restore_step:
            optim.load_state_dict(ckpt["optimizer"])
        model.train()
        return model, optim
    model.eval()
    model.requires_grad_ = False  # (sic) the reference sets an attribute, not requires_grad_()
    return model


def get_param_num(model):
    """utils/model.py:37-39."""
    return sum(p.numel() for p in model.parameters())
