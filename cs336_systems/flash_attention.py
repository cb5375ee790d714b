"""Reference-path module (``cs336_systems/flash_attention.py``): FlashAttentionTorch and the GPU
FlashAttention class. ``FlashAttentionTriton`` is kept as a name for the adapter contract; it is
the hand-written HIP implementation (no Triton anywhere)."""

from .ops.flash_attention import (  # noqa: F401
    FlashAttentionHIP,
    FlashAttentionTorch,
    FlashAttentionTriton,
    flash_attention,
    naive_attention,
)
