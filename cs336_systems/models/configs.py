"""Model-size registry (``cs336_systems/benchmark.py:247-259`` of the reference; handout Table 1).

Parameter counts (vocab 10000, untied head, SwiGLU with three matrices) are computed exactly by
:func:`param_count`; e.g. ``xl`` ≈ 2.00 B, ``2.7b`` ≈ 3.41 B.
"""

from __future__ import annotations

MODEL_CONFIGS: dict[str, dict[str, int]] = {
    "small": dict(d_model=768, d_ff=3072, num_layers=12, num_heads=12),
    "medium": dict(d_model=1024, d_ff=4096, num_layers=24, num_heads=16),
    "large": dict(d_model=1280, d_ff=5120, num_layers=36, num_heads=20),
    "xl": dict(d_model=1600, d_ff=6400, num_layers=48, num_heads=25),
    "2.7b": dict(d_model=2560, d_ff=10240, num_layers=32, num_heads=32),
    # tiny config for tests / smoke runs
    "tiny": dict(d_model=128, d_ff=384, num_layers=2, num_heads=2),
}

DEFAULT_VOCAB = 10000
DEFAULT_THETA = 10000.0


def get_model_config(model_size: str) -> dict[str, int]:
    try:
        return dict(MODEL_CONFIGS[model_size])
    except KeyError:
        raise ValueError(f"Unknown model size: {model_size}") from None


def param_count(model_size: str, vocab_size: int = DEFAULT_VOCAB) -> int:
    c = MODEL_CONFIGS[model_size]
    d, f, L = c["d_model"], c["d_ff"], c["num_layers"]
    per_layer = 4 * d * d + 3 * d * f + 2 * d
    return 2 * vocab_size * d + L * per_layer + d


def train_flops_per_token(model_size: str, context_length: int, vocab_size: int = DEFAULT_VOCAB, causal: bool = True) -> float:
    """6*N_matmul_params + attention (QK^T and PV: 2 GEMMs * 2 flops * 3 (fwd+bwd) per layer)."""
    c = MODEL_CONFIGS[model_size]
    d, f, L = c["d_model"], c["d_ff"], c["num_layers"]
    matmul_params = L * (4 * d * d + 3 * d * f) + vocab_size * d
    attn = L * 12 * context_length * d * (0.5 if causal else 1.0)
    return 6.0 * matmul_params + attn
