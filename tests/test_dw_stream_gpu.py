"""Weight-gradient GEMMs on the side stream (models/fused.py): gradients are bitwise identical to
the single-stream run, the main stream is synchronized by the end of backward, and accumulation
into existing grads (which must not use the side stream) still matches."""

import pytest
import torch

from cs336_systems import ops
from cs336_systems.models import BasicsTransformerLM
from cs336_systems.models import fused

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _run(model, x, y, accumulate=False):
    if not accumulate:
        model.zero_grad(set_to_none=True)
    with torch.autocast("cuda", dtype=torch.bfloat16):
        loss = ops.cross_entropy(model(x), y)
    loss.backward()
    # consume the grads on the main stream right away (no explicit synchronize)
    return {n: p.grad.clone() for n, p in model.named_parameters()}


@pytest.mark.parametrize("accumulate", [False, True])
def test_side_stream_dw_matches(monkeypatch, accumulate):
    torch.manual_seed(0)
    model = BasicsTransformerLM(vocab_size=512, context_length=128, d_model=256, num_layers=3, num_heads=4, d_ff=768, device=DEV)
    x = torch.randint(0, 512, (8, 128), device=DEV)
    y = torch.randint(0, 512, (8, 128), device=DEV)
    monkeypatch.setenv("CS336_DW_STREAM", "0")
    ref = _run(model, x, y)
    if accumulate:
        ref2 = _run(model, x, y, accumulate=True)
    monkeypatch.setenv("CS336_DW_STREAM", "1")
    got = _run(model, x, y)
    assert not fused._state["dirty"], "end-of-backward callback did not synchronize"
    for n in ref:
        torch.testing.assert_close(got[n], ref[n], rtol=0, atol=0, msg=n)
    if accumulate:
        got2 = _run(model, x, y, accumulate=True)
        for n in ref2:
            torch.testing.assert_close(got2[n], ref2[n], rtol=0, atol=0, msg=n)
