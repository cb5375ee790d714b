"""Rotary position embedding (interleaved pairs), eager reference + HIP kernel.

Reference semantics (``cs336-basics/cs336_basics/model.py:113-147``): the cache holds
``cos/sin(t * theta^(-2i/d))`` of shape ``(2, ctx, d/2)``; pairs ``(x[2i], x[2i+1])`` are rotated by
angle ``t * f_i`` with ``t`` the token position.

HIP path (``csrc/ops/rope.hip``): ``x`` is a 4-D ``(B, H, N, D)`` view with any batch/head/seq
strides (typically a transposed view of a ``(B, N, H, D)`` projection output, so no transpose copy
is ever made); the output is written in ``(B, N, H, D)`` memory order and returned as the
``(B, H, N, D)`` view that the flash-attention kernels consume directly. Backward is the same
kernel with the inverse rotation.
"""

from __future__ import annotations

import torch

from ._ext import ops, use_hip


def rope_ref(x: torch.Tensor, cos: torch.Tensor, sin: torch.Tensor, pos: torch.Tensor) -> torch.Tensor:
    """``x``: (..., seq, d); ``cos``/``sin``: (ctx, d/2); ``pos``: int positions broadcastable to x[..., 0]."""
    x1 = x[..., 0::2]
    x2 = x[..., 1::2]
    c = cos[pos].to(x.dtype) if x.dtype != torch.float32 else cos[pos]
    s = sin[pos].to(x.dtype) if x.dtype != torch.float32 else sin[pos]
    r1 = c * x1 - s * x2
    r2 = s * x1 + c * x2
    return torch.stack((r1, r2), dim=-1).flatten(-2).contiguous()


class RoPEHIP(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, cos, sin, pos):
        ctx.save_for_backward(cos, sin, pos)
        return ops().rope(x, cos, sin, pos, False)

    @staticmethod
    def backward(ctx, dy):
        cos, sin, pos = ctx.saved_tensors
        return ops().rope(dy, cos, sin, pos, True), None, None, None


def _normalize_pos(pos: torch.Tensor | None, B: int, N: int) -> torch.Tensor | None:
    if pos is None:
        return None
    p = pos
    while p.dim() > 2:  # (..., 1, seq) style broadcast positions from the reference module
        if p.shape[-2] != 1:
            return "general"  # type: ignore[return-value]
        p = p.squeeze(-2)
    if p.dim() == 1:
        p = p.unsqueeze(0)
    if p.shape[-1] != N or p.shape[0] not in (1, B):
        return "general"  # type: ignore[return-value]
    return p.expand(B, N).to(torch.int64).contiguous()


def _hip_layout_ok(x: torch.Tensor) -> bool:
    """The kernel moves 16 B per access: contiguous last dim, head dim a multiple of 8 in [8, 256],
    16-byte aligned base and strides (the fused-QKV slices and fresh tensors always are)."""
    D, es = x.shape[-1], x.element_size()
    return (
        x.stride(-1) == 1
        and 8 <= D <= 256
        and D % 8 == 0
        and x.data_ptr() % 16 == 0
        and all((x.stride(i) * es) % 16 == 0 for i in range(3))
    )


def rope(x: torch.Tensor, cos: torch.Tensor, sin: torch.Tensor, pos: torch.Tensor | None = None) -> torch.Tensor:
    """Apply RoPE to ``x`` of shape (..., seq, d)."""
    if x.dim() == 4 and use_hip(x) and _hip_layout_ok(x):
        B, H, N, D = x.shape
        p = _normalize_pos(pos, B, N)
        if not isinstance(p, str):
            return RoPEHIP.apply(x, cos.float().contiguous(), sin.float().contiguous(), p)
    if pos is None:
        pos = torch.arange(x.shape[-2], device=x.device)
    return rope_ref(x, cos, sin, pos)
