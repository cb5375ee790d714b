"""SwiGLU gate ``silu(a) * b`` (``cs336-basics/cs336_basics/model.py:389-397, 526-527``).

The HIP kernel (``csrc/ops/swiglu.hip``) fuses sigmoid, the two multiplies and the dtype cast into
one vectorized pass (8 bf16 per lane), and the backward produces ``da`` and ``db`` in one pass
from ``(dh, a, b)`` instead of the ~6 eager kernels autograd would launch.
"""

from __future__ import annotations

import torch

from ._ext import ops, use_hip


def silu(x: torch.Tensor) -> torch.Tensor:
    return x * torch.sigmoid(x)


def silu_mul_ref(a: torch.Tensor, b: torch.Tensor) -> torch.Tensor:
    return silu(a) * b


class SiluMulHIP(torch.autograd.Function):
    @staticmethod
    def forward(ctx, a, b):
        a = a.contiguous()
        b = b.contiguous()
        ctx.save_for_backward(a, b)
        return ops().silu_mul_fwd(a, b)

    @staticmethod
    def backward(ctx, dh):
        a, b = ctx.saved_tensors
        da, db = ops().silu_mul_bwd(dh.contiguous(), a, b)
        return da, db


def silu_mul(a: torch.Tensor, b: torch.Tensor) -> torch.Tensor:
    if a.shape == b.shape and a.dtype == b.dtype and use_hip(a, b):
        return SiluMulHIP.apply(a, b)
    return silu_mul_ref(a, b)
