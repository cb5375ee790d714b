"""Re-export of the model layers (reference ``cs336-basics/cs336_basics/model.py``)."""

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
)

from .nn_utils import softmax  # noqa: F401
