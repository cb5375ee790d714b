"""Whole-step HIP graph (utils/graphs.py GraphedTrainStep): zero grads, forward,
loss, backward and the fused AdamW update -- plain or overlapped with the backward on a side
stream -- captured once and replayed on new batches. The bias correction comes from a device-side
step counter (FusedAdamW.enable_device_step), so five replays with different batches must equal
five eager steps BIT FOR BIT: losses, parameters, optimizer state and bf16 / Wᵀ shadows. Also:
the device-step update alone equals the host-scalar update, and the deterministic embedding
backward (csrc/ops/embedding.hip) against an fp64 reference."""

import pytest
import torch

from cs336_systems import ops
from cs336_systems.models import BasicsTransformerLM
from cs336_systems.models.fused import get_shadow, get_shadow_t
from cs336_systems.utils.graphs import GraphedTrainStep

pytestmark = pytest.mark.gpu
DEV = "cuda"
V, CTX = 512, 64


def _setup(overlap):
    torch.manual_seed(0)
    model = BasicsTransformerLM(vocab_size=V, context_length=CTX, d_model=256, num_layers=3, num_heads=4, d_ff=768, device=DEV)
    opt = ops.FusedAdamW(model.parameters(), lr=1e-3, betas=(0.9, 0.95), weight_decay=0.1, bf16_shadows=True)
    if overlap:
        assert opt.enable_backward_overlap(chunk_mb=1.0)

    def step(x, y):
        opt.zero_grad(set_to_none=True)
        with torch.autocast("cuda", dtype=torch.bfloat16):
            loss = ops.cross_entropy(model(x), y)
        loss.backward()
        opt.step()
        return loss

    return model, opt, step


def _batches(n):
    g = torch.Generator(device=DEV).manual_seed(7)
    return [torch.randint(0, V, (4, CTX + 1), device=DEV, generator=g) for _ in range(n)]


def _same(a, b, what):
    assert torch.equal(a, b), f"{what}: max |diff| {(a.float() - b.float()).abs().max().item()}"


@pytest.mark.parametrize("overlap", [False, True])
def test_graphed_train_step_bitwise_equals_eager(overlap):
    bs = _batches(7)
    ref, ref_opt, ref_step = _setup(overlap)
    ref_losses = []
    for t in bs:
        ref_losses.append(ref_step(t[:, :-1], t[:, 1:]).detach().clone())
    torch.cuda.synchronize()

    model, opt, step = _setup(overlap)
    step(bs[0][:, :-1], bs[0][:, 1:])  # eager step 1: creates the optimizer state
    g = GraphedTrainStep(step, opt, bs[1][:, :-1], bs[1][:, 1:], warmup=1)  # real step 2 + capture
    losses = []
    for t in bs[2:]:  # five replays, each on a new batch
        losses.append(g(t[:, :-1], t[:, 1:]).detach().clone())
    torch.cuda.synchronize()

    for i, (a, b) in enumerate(zip(losses, ref_losses[2:])):
        _same(a, b, f"loss of step {i + 3}")
    assert opt.device_step_value() == len(bs)
    for (n, a), b in zip(model.named_parameters(), ref.parameters()):
        _same(a, b, n)
        sa, sb = opt.state[a], ref_opt.state[b]
        assert sa["t"] == sb["t"] == len(bs) + 1, (n, sa["t"], sb["t"])
        _same(sa["m"], sb["m"], n + " m")
        _same(sa["v"], sb["v"], n + " v")
        if get_shadow(a) is not None:
            _same(get_shadow(a), get_shadow(b), n + " shadow")
        if get_shadow_t(a) is not None and get_shadow_t(b) is not None:
            _same(get_shadow_t(a), get_shadow_t(b), n + " shadow_t")


def test_device_step_update_equals_host_scalar():
    """Eager steps with the device-side step counter give the host-scalar result bit for bit (the
    step size is the same double expression rounded once to fp32)."""
    bs = _batches(6)
    ref, ref_opt, ref_step = _setup(False)
    model, opt, step = _setup(False)
    for i, t in enumerate(bs):
        ref_step(t[:, :-1], t[:, 1:])
        step(t[:, :-1], t[:, 1:])
        if i == 0:
            opt.enable_device_step()
    torch.cuda.synchronize()
    assert opt.device_step_value() == len(bs)
    for (n, a), b in zip(model.named_parameters(), ref.parameters()):
        _same(a, b, n)


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
def test_embedding_backward_matches_fp64_and_repeats(dt):
    torch.manual_seed(3)
    Vb, D, T = 1000, 96, 4096
    ids = torch.randint(0, Vb // 2, (T,), device=DEV)  # half the rows never occur: written as zeros
    ids[:300] = 7  # one long run
    g = torch.randn(T, D, device=DEV).to(dt)
    s, perm = torch.sort(ids, stable=True)
    gw = torch.ops.cs336.embedding_bwd(g, s, perm, Vb)
    ref = torch.zeros(Vb, D, dtype=torch.float64, device=DEV).index_add_(0, ids, g.double())
    torch.testing.assert_close(gw.double(), ref, rtol=1e-5, atol=1e-5)
    out = torch.full((Vb, D), float("nan"), device=DEV)
    torch.ops.cs336.embedding_bwd_into(g, s, perm, out)
    _same(out, gw, "into vs fresh")
    _same(torch.ops.cs336.embedding_bwd(g, s, perm, Vb), gw, "repeat")


def test_embedding_module_backward_deterministic():
    torch.manual_seed(4)
    emb = torch.nn.Embedding(10000, 1600, device=DEV)
    from cs336_systems.models.transformer import Embedding

    m = Embedding(10000, 1600, device=DEV)
    ids = torch.randint(0, 10000, (8, 512), device=DEV)
    grads = []
    for _ in range(2):
        m.weight.grad = None
        m(ids).pow(2).sum().backward()
        grads.append(m.weight.grad.clone())
    _same(grads[0], grads[1], "two backward passes")
    emb.weight.data.copy_(m.weight.data)
    emb(ids).pow(2).sum().backward()
    torch.testing.assert_close(grads[0], emb.weight.grad, rtol=1e-5, atol=1e-4)
