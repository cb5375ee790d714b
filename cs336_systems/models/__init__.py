from .configs import DEFAULT_THETA, DEFAULT_VOCAB, MODEL_CONFIGS, get_model_config, param_count, train_flops_per_token
from .transformer import (
    BasicsTransformerLM,
    CausalMultiHeadSelfAttention,
    Embedding,
    Linear,
    RMSNorm,
    RotaryEmbedding,
    SwiGLU,
    TransformerBlock,
    get_attention_impl,
    scaled_dot_product_attention,
    set_attention_impl,
    silu,
    softmax,
)


def build_model(size: str, context_length: int, vocab_size: int = DEFAULT_VOCAB, rope_theta: float = DEFAULT_THETA, device=None, dtype=None, fused_layout: bool = True):
    """Construct a :class:`BasicsTransformerLM` of a registry size directly on ``device``."""
    cfg = get_model_config(size)
    return BasicsTransformerLM(
        vocab_size=vocab_size, context_length=context_length, rope_theta=rope_theta, device=device, dtype=dtype, fused_layout=fused_layout, **cfg
    )


__all__ = [
    "BasicsTransformerLM",
    "CausalMultiHeadSelfAttention",
    "Embedding",
    "Linear",
    "RMSNorm",
    "RotaryEmbedding",
    "SwiGLU",
    "TransformerBlock",
    "MODEL_CONFIGS",
    "DEFAULT_VOCAB",
    "DEFAULT_THETA",
    "build_model",
    "get_model_config",
    "param_count",
    "train_flops_per_token",
    "get_attention_impl",
    "set_attention_impl",
    "scaled_dot_product_attention",
    "silu",
    "softmax",
]
