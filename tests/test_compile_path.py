"""torch.compile path of the model (models/compiled.py custom ops) on CPU: the whole train step
(forward, loss, backward) traces with no graph break under bf16 autocast, and the compiled step's
loss and gradients match the eager model's. On CPU the custom ops run their reference math; the GPU
twin (tests/test_compile_gpu.py) runs the HIP kernels."""

import pytest
import torch

from cs336_systems import ops
from cs336_systems.models import transformer
from cs336_systems.models.transformer import BasicsTransformerLM


@pytest.fixture
def cpu_ops(monkeypatch):
    monkeypatch.setattr(transformer, "_COMPILE_CPU_OPS", True)
    torch._dynamo.reset()
    yield
    torch._dynamo.reset()


def _model():
    torch.manual_seed(0)
    return BasicsTransformerLM(vocab_size=97, context_length=32, d_model=64, num_layers=2, num_heads=4, d_ff=160)


def _step(model, x):
    with torch.autocast("cpu", dtype=torch.bfloat16):
        logits = model(x)
    return ops.cross_entropy(logits.float(), x)


def test_compiled_step_has_no_graph_break(cpu_ops):
    model = _model()
    x = torch.randint(0, 97, (2, 32))
    ex = torch._dynamo.explain(lambda x: _step(model, x))(x)
    assert ex.graph_break_count == 0, ex.break_reasons
    assert ex.graph_count == 1


def test_compiled_step_matches_eager(cpu_ops):
    model = _model()
    ref = _model()
    ref.load_state_dict(model.state_dict())
    x = torch.randint(0, 97, (2, 32))
    step = torch.compile(lambda x: _step(model, x), backend="aot_eager", fullgraph=True)
    loss = step(x)
    loss.backward()
    transformer._COMPILE_CPU_OPS = False  # the eager reference model takes the plain module path
    loss_ref = _step(ref, x)
    loss_ref.backward()
    assert torch.allclose(loss.float(), loss_ref.float(), rtol=2e-2, atol=2e-2), (loss.item(), loss_ref.item())
    for (n, p), (_, q) in zip(model.named_parameters(), ref.named_parameters()):
        assert p.grad is not None, n
        err = (p.grad - q.grad).norm() / (q.grad.norm() + 1e-12)
        assert err < 5e-2, (n, float(err))
