"""Student ``cs336_basics.transformer`` API imported by the reference's systems code
(``benchmark.py:3``, ``naive_ddp.py:10``), absent from the reference repo.

``TransformerLM(d_model, num_heads, d_ff, vocab_size, context_length, num_layers, max_seq_len=None,
theta=None, device=None, dtype=None)`` with submodules ``token_embeddings``,
``layers[i].{ln1, attn, ln2, ffn}``, ``ln_final``, ``lm_head`` (state-dict keys such as
``layers.1.ln1.weight`` match, ``naive_ddp.py:263``).
"""

from __future__ import annotations

import torch

from cs336_systems.models.transformer import (  # noqa: F401
    BasicsTransformerLM,
    CausalMultiHeadSelfAttention,
    Embedding,
    Linear,
    RMSNorm,
    RotaryEmbedding,
    SwiGLU,
    TransformerBlock,
    scaled_dot_product_attention,
    silu,
    softmax,
)

RoPE = RotaryEmbedding
SwiGLUFeedForward = SwiGLU
MultiHeadSelfAttention = CausalMultiHeadSelfAttention


class TransformerLM(BasicsTransformerLM):
    def __init__(
        self,
        d_model: int,
        num_heads: int,
        d_ff: int,
        vocab_size: int,
        context_length: int,
        num_layers: int,
        max_seq_len: int | None = None,
        theta: float | None = None,
        device=None,
        dtype=None,
    ):
        super().__init__(
            vocab_size=vocab_size,
            context_length=max(context_length, max_seq_len or 0),
            d_model=d_model,
            num_layers=num_layers,
            num_heads=num_heads,
            d_ff=d_ff,
            rope_theta=10000.0 if theta is None else theta,
            device=device,
            dtype=dtype,
        )
        if device is not None or dtype is not None:
            self.to(device=device, dtype=dtype)
