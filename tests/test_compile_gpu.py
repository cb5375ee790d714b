"""torch.compile of the Transformer on the HIP path (models/compiled.py custom ops): no graph break
for the XL and 2.7b models under bf16 autocast, and a compiled train step (inductor) that matches the
eager step -- loss, gradients, and the parameters after fused-AdamW steps, with and without the bf16 /
Wᵀ weight shadows that the fused AdamW writes and the custom ops read."""

import pytest
import torch

from cs336_systems import ops
from cs336_systems.models import build_model
from cs336_systems.models.transformer import BasicsTransformerLM

pytestmark = pytest.mark.gpu


def _ext():
    if not torch.cuda.is_available():
        pytest.skip("needs a GPU")
    assert ops.load_ext(), ops.load_error()


@pytest.mark.parametrize("size", ["xl", "2.7b"])
def test_no_graph_break(size):
    _ext()
    torch._dynamo.reset()
    dev = torch.device("cuda", 0)
    model = build_model(size, 512, device=dev)
    x = torch.randint(0, 10000, (1, 512), device=dev)

    def step(x):
        with torch.autocast("cuda", dtype=torch.bfloat16):
            return ops.cross_entropy(model(x), x)

    ex = torch._dynamo.explain(step)(x)
    assert ex.graph_break_count == 0, ex.break_reasons
    assert ex.graph_count == 1
    del model
    torch.cuda.empty_cache()
    torch._dynamo.reset()


def _small(dev):
    torch.manual_seed(0)
    return BasicsTransformerLM(vocab_size=10000, context_length=256, d_model=640, num_layers=2, num_heads=10, d_ff=2560,
                               device=dev)


@pytest.mark.parametrize("shadows", [False, True])
def test_compiled_steps_match_eager(shadows):
    _ext()
    torch._dynamo.reset()
    dev = torch.device("cuda", 0)
    mc, me = _small(dev), _small(dev)
    me.load_state_dict(mc.state_dict())
    kw = dict(lr=1e-3, betas=(0.9, 0.95), eps=1e-8, weight_decay=0.01)
    kw["bf16_shadows"] = shadows
    oc, oe = ops.FusedAdamW(mc.parameters(), **kw), ops.FusedAdamW(me.parameters(), **kw)
    x = torch.randint(0, 10000, (2, 256), device=dev)

    def loss_of(m):
        with torch.autocast("cuda", dtype=torch.bfloat16):
            return ops.cross_entropy(m(x), x)

    cstep = torch.compile(lambda: loss_of(mc), fullgraph=True)
    for it in range(3):
        oc.zero_grad(set_to_none=True)
        oe.zero_grad(set_to_none=True)
        lc, le = cstep(), loss_of(me)
        lc.backward()
        le.backward()
        assert torch.allclose(lc.float(), le.float(), rtol=1e-2, atol=1e-2), (it, lc.item(), le.item())
        for (n, p), (_, q) in zip(mc.named_parameters(), me.named_parameters()):
            err = (p.grad - q.grad).norm() / (q.grad.norm() + 1e-12)
            assert err < 3e-2, (it, n, float(err))
        oc.step()
        oe.step()
    for (n, p), (_, q) in zip(mc.named_parameters(), me.named_parameters()):
        # Adam normalizes each update to ~lr, so bf16-level gradient differences can move a weight by up to
        # lr per step: compare against 4 lr after the 3 steps
        assert (p - q).abs().max().item() <= 4e-3, (n, (p - q).abs().max().item())
    torch._dynamo.reset()
