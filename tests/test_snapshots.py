"""Pinned numerics (snapshot fixtures): the pure-PyTorch tiled FA2 (forward O/L, causal and not) and
a seeded small LM's logits/loss on CPU are compared against committed ``tests/_snapshots/*.npz`` —
a regression net for the reference path that every HIP kernel is tested against."""

import torch

from cs336_systems.models import BasicsTransformerLM
from cs336_systems.ops.flash_attention import FlashAttentionTorch


def test_flash_torch_snapshot(numpy_snapshot):
    g = torch.Generator().manual_seed(7)
    q, k, v = (torch.randn(2, 48, 32, generator=g) for _ in range(3))
    out = {}
    for causal in (False, True):
        o = FlashAttentionTorch.apply(q, k, v, causal)
        out[f"o_causal{int(causal)}"] = o
    numpy_snapshot.assert_match(out, "flash_torch")


def test_small_lm_snapshot(numpy_snapshot):
    torch.manual_seed(3)
    model = BasicsTransformerLM(vocab_size=64, context_length=32, d_model=32, num_layers=2, num_heads=2, d_ff=64)
    x = torch.randint(0, 64, (2, 32), generator=torch.Generator().manual_seed(5))
    with torch.no_grad():
        logits = model(x)
    loss = torch.nn.functional.cross_entropy(logits.reshape(-1, 64), x.reshape(-1))
    numpy_snapshot.assert_match({"logits": logits, "loss": loss}, "small_lm", rtol=1e-4, atol=1e-5)
