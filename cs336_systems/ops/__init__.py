"""Kernel layer: every hot op has an eager PyTorch reference (used on CPU and as the numerics
oracle in tests) and a hand-written HIP/CDNA4 kernel (used for GPU tensors)."""

from ._ext import backend, ext_available, get_backend, load_error, load_ext, set_backend, use_hip
from .adamw import FusedAdamW, clip_grad_norm_, multi_tensor_l2norm
from .cross_entropy import cross_entropy, cross_entropy_ref
from .flash_attention import (
    FlashAttentionHIP,
    FlashAttentionTorch,
    FlashAttentionTriton,
    flash_attention,
    naive_attention,
)
from .rmsnorm import add_rmsnorm, add_rmsnorm_ref, rmsnorm, rmsnorm_ref
from .rope import rope, rope_ref
from .swiglu import silu, silu_mul, silu_mul_ref

__all__ = [
    "backend",
    "ext_available",
    "get_backend",
    "load_error",
    "load_ext",
    "set_backend",
    "use_hip",
    "FusedAdamW",
    "clip_grad_norm_",
    "multi_tensor_l2norm",
    "cross_entropy",
    "cross_entropy_ref",
    "FlashAttentionHIP",
    "FlashAttentionTorch",
    "FlashAttentionTriton",
    "flash_attention",
    "naive_attention",
    "add_rmsnorm",
    "add_rmsnorm_ref",
    "rmsnorm",
    "rmsnorm_ref",
    "rope",
    "rope_ref",
    "silu",
    "silu_mul",
    "silu_mul_ref",
]
