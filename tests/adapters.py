"""Adapter contract of the reference test suite (``tests/adapters.py``), bound to the MI355X
implementations. Function names and signatures are unchanged."""

from __future__ import annotations

from typing import Type

import torch

from cs336_systems.ops.flash_attention import FlashAttentionHIP, FlashAttentionTorch
from cs336_systems.parallel.ddp import DDPBucketed, DDPIndividual
from cs336_systems.parallel.sharded_optimizer import ShardedOptimizer


def get_flashattention_autograd_function_pytorch() -> Type:
    """Tiled FlashAttention-2 in plain PyTorch (autograd.Function class)."""
    return FlashAttentionTorch


def get_flashattention_autograd_function_triton() -> Type:
    """The GPU-kernel FlashAttention-2 class: hand-written HIP/CDNA4 kernels on MI355X."""
    return FlashAttentionHIP


def get_ddp_individual_parameters(module: torch.nn.Module) -> torch.nn.Module:
    return DDPIndividual(module)


def ddp_individual_parameters_on_after_backward(ddp_model: torch.nn.Module, optimizer: torch.optim.Optimizer):
    ddp_model.finish_gradient_synchronization()


def get_ddp_bucketed(module: torch.nn.Module, bucket_size_mb: float) -> torch.nn.Module:
    return DDPBucketed(module, bucket_size_mb=bucket_size_mb)


def ddp_bucketed_on_after_backward(ddp_model: torch.nn.Module, optimizer: torch.optim.Optimizer):
    ddp_model.finish_gradient_synchronization()


def ddp_bucketed_on_train_batch_start(ddp_model: torch.nn.Module, optimizer: torch.optim.Optimizer):
    ddp_model.on_train_batch_start()


def get_sharded_optimizer(params, optimizer_cls: Type[torch.optim.Optimizer], **kwargs) -> torch.optim.Optimizer:
    return ShardedOptimizer(params, optimizer_cls, **kwargs)
