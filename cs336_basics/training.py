"""Student ``cs336_basics.training`` API (``benchmark.py:5``): loss, clipping, batches, checkpoints."""

from __future__ import annotations

import os
import typing

import torch

from cs336_systems import ops as _ops
from cs336_systems.data import get_batch  # noqa: F401


def cross_entropy_loss(inputs: torch.Tensor, targets: torch.Tensor) -> torch.Tensor:
    """Mean cross-entropy of logits ``(..., V)`` against int targets ``(...)``."""
    return _ops.cross_entropy(inputs, targets)


def gradient_clipping(parameters, max_l2_norm: float) -> torch.Tensor:
    return _ops.clip_grad_norm_(list(parameters), max_l2_norm)


def save_checkpoint(model: torch.nn.Module, optimizer: torch.optim.Optimizer, iteration: int, out: str | os.PathLike | typing.BinaryIO) -> None:
    torch.save({"model": model.state_dict(), "optimizer": optimizer.state_dict(), "iteration": iteration}, out)


def load_checkpoint(src, model: torch.nn.Module, optimizer: torch.optim.Optimizer | None = None) -> int:
    ckpt = torch.load(src, weights_only=True, map_location="cpu")
    model.load_state_dict(ckpt["model"])
    if optimizer is not None:
        optimizer.load_state_dict(ckpt["optimizer"])
    return int(ckpt["iteration"])
