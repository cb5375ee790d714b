"""HIP-graph captured training step (utils/graphs.py): replaying the captured forward + backward
with fresh batches and stepping FusedAdamW eagerly reproduces the eager training run (losses and
parameters); the e2e benchmark's --graphs mode runs."""

import pytest
import torch

from cs336_systems import ops
from cs336_systems.bench import e2e
from cs336_systems.models import BasicsTransformerLM
from cs336_systems.utils.graphs import GraphedStep

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _model():
    torch.manual_seed(0)
    return BasicsTransformerLM(vocab_size=512, context_length=128, d_model=256, num_layers=2, num_heads=4, d_ff=768, device=DEV)


def _batches(n):
    g = torch.Generator(device=DEV).manual_seed(3)
    return [torch.randint(0, 512, (4, 129), device=DEV, generator=g) for _ in range(n)]


def _loss(model):
    def f(x, y):
        with torch.autocast("cuda", dtype=torch.bfloat16):
            return ops.cross_entropy(model(x), y)

    return f


def test_graphed_step_matches_eager():
    batches = _batches(4)
    ref = _model()
    opt_r = ops.FusedAdamW(ref.parameters(), lr=1e-3, bf16_shadows=True)
    losses_r = []
    for t in batches:
        opt_r.zero_grad(set_to_none=True)
        loss = _loss(ref)(t[:, :-1], t[:, 1:])
        loss.backward()
        opt_r.step()
        losses_r.append(loss.item())
    model = _model()
    opt = ops.FusedAdamW(model.parameters(), lr=1e-3, bf16_shadows=True)
    step = GraphedStep(_loss(model), model.parameters(), batches[0][:, :-1], batches[0][:, 1:])
    losses = []
    for t in batches:
        loss = step(t[:, :-1], t[:, 1:])
        opt.step()
        losses.append(loss.item())
    torch.testing.assert_close(torch.tensor(losses), torch.tensor(losses_r), rtol=1e-5, atol=1e-5)
    for (n, a), b in zip(model.named_parameters(), ref.parameters()):
        torch.testing.assert_close(a, b, rtol=1e-5, atol=1e-6, msg=n)


def test_graph_replay_with_different_token_sets():
    """Captured on a batch with one distinct token, replayed on random batches: the embedding
    backward inside the graph must not depend on the captured batch's token set (ATen's sort/
    partition-based embedding backward faulted here at the XL shape)."""
    torch.manual_seed(0)
    model = BasicsTransformerLM(vocab_size=10000, context_length=256, d_model=128, num_layers=1, num_heads=2, d_ff=256, device=DEV)
    x0 = torch.zeros(16, 256, dtype=torch.long, device=DEV)
    step = GraphedStep(_loss(model), model.parameters(), x0, x0)
    for i in range(3):
        t = torch.randint(0, 10000, (16, 257), device=DEV)
        loss = step(t[:, :-1], t[:, 1:])
        g = model.token_embeddings.weight.grad.clone()
        model.zero_grad(set_to_none=True)
        ref = _loss(model)(t[:, :-1], t[:, 1:])
        ref.backward()
        torch.testing.assert_close(loss, ref.detach(), rtol=1e-5, atol=1e-5)
        torch.testing.assert_close(g, model.token_embeddings.weight.grad, rtol=1e-4, atol=1e-6)
    torch.cuda.synchronize()


def test_e2e_benchmark_graphs_mode():
    row = e2e.run_simple_benchmark("small", 128, 2, warmup_steps=2, timed_steps=3, mixed_precision=True, graphs=True)
    assert row["graphs"] and row["step_ms"] > 0


def test_train_driver_graphs(tmp_path):
    from cs336_systems.train import TrainConfig, train

    import os

    os.environ.update(RANK="0", WORLD_SIZE="1", LOCAL_RANK="0", MASTER_ADDR="127.0.0.1")
    from cs336_systems.parallel.comm import cleanup_distributed, find_free_port

    os.environ["MASTER_PORT"] = str(find_free_port())
    cfg = TrainConfig(size="tiny", ctx=64, vocab=500, batch=4, steps=4, warmup=1, lr=1e-3, clip=1.0, graphs=True,
                      device="cuda", log_every=1, ckpt_dir=str(tmp_path / "ck"))
    try:
        out = train(cfg)
    finally:
        cleanup_distributed()
    losses = [h["loss"] for h in out["history"]]
    assert len(losses) == 4 and all(0 < v < 10 for v in losses)
