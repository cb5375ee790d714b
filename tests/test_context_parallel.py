"""Context parallelism (parallel/context_parallel.py) on CPU/gloo: ring attention over 2 and 4 ranks
matches full attention (outputs and q/k/v gradients) for both sequence layouts, causal and not, and
a context-parallel Transformer LM step (loss and DP-averaged gradients) matches the single-process
model on the whole sequence."""

import os

import pytest
import torch
import torch.distributed as dist

from cs336_systems.models import BasicsTransformerLM
from cs336_systems.ops.flash_attention import naive_attention
from cs336_systems.parallel import (
    enable_context_parallel,
    ring_attention,
    sequence_positions,
    shard_sequence,
    ulysses_attention,
    unshard_sequence,
)

from .common import spawn


def _init(rank, world):
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world))
    dist.init_process_group("gloo", rank=rank, world_size=world)


def _attn_worker(rank, world, layout, causal):
    _init(rank, world)
    torch.manual_seed(0)
    B, H, N, D = 2, 3, 8 * world, 16
    q, k, v, do = (torch.randn(B, H, N, D, dtype=torch.float64) for _ in range(4))
    qf, kf, vf = (t.clone().requires_grad_(True) for t in (q, k, v))
    of = naive_attention(qf, kf, vf, is_causal=causal)
    of.backward(do)
    sh = lambda t: shard_sequence(t, rank, world, layout, dim=2)  # noqa: E731
    ql, kl, vl = (sh(t).requires_grad_(True) for t in (q, k, v))
    ol = ring_attention(ql, kl, vl, None, causal, layout)
    ol.backward(sh(do))
    # the tiled CPU kernels accumulate in fp32
    tol = dict(rtol=1e-5, atol=1e-5)
    torch.testing.assert_close(ol, sh(of.detach()), **tol)
    for got, ref in ((ql, qf), (kl, kf), (vl, vf)):
        torch.testing.assert_close(got.grad, sh(ref.grad), **tol)
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 4])
@pytest.mark.parametrize("layout", ["contiguous", "zigzag"])
@pytest.mark.parametrize("causal", [True, False])
def test_ring_attention_matches_full(world, layout, causal):
    spawn(_attn_worker, world, layout, causal)


def _ulysses_worker(rank, world, causal):
    _init(rank, world)
    torch.manual_seed(0)
    B, H, N, D = 2, 2 * world, 8 * world, 16
    q, k, v, do = (torch.randn(B, H, N, D, dtype=torch.float64) for _ in range(4))
    qf, kf, vf = (t.clone().requires_grad_(True) for t in (q, k, v))
    naive_attention(qf, kf, vf, is_causal=causal).backward(do)
    of = naive_attention(q, k, v, is_causal=causal)
    sh = lambda t: shard_sequence(t, rank, world, "ulysses", dim=2)  # noqa: E731
    ql, kl, vl = (sh(t).requires_grad_(True) for t in (q, k, v))
    ol = ulysses_attention(ql, kl, vl, None, causal)
    ol.backward(sh(do))
    tol = dict(rtol=1e-10, atol=1e-10)  # the same fp64 math, only re-distributed
    torch.testing.assert_close(ol, sh(of), **tol)
    for got, ref in ((ql, qf), (kl, kf), (vl, vf)):
        torch.testing.assert_close(got.grad, sh(ref.grad), **tol)
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 4])
@pytest.mark.parametrize("causal", [True, False])
def test_ulysses_attention_matches_full(world, causal):
    spawn(_ulysses_worker, world, causal)


def test_shard_roundtrip_and_positions():
    x = torch.arange(2 * 24).view(2, 24)
    for layout in ("contiguous", "zigzag"):
        parts = [shard_sequence(x, r, 3, layout) for r in range(3)]
        assert torch.equal(unshard_sequence(parts, layout), x)
        pos = torch.cat([sequence_positions(24, r, 3, layout) for r in range(3)])
        assert sorted(pos.tolist()) == list(range(24))
    assert sequence_positions(8, 0, 2, "zigzag").tolist() == [0, 1, 6, 7]


CFG = dict(vocab_size=97, context_length=32, d_model=64, num_layers=2, num_heads=4, d_ff=96)


def _model_worker(rank, world, layout):
    _init(rank, world)
    torch.manual_seed(0)
    ref = BasicsTransformerLM(**CFG).double()
    model = BasicsTransformerLM(**CFG).double()
    model.load_state_dict(ref.state_dict())
    enable_context_parallel(model, None, layout)
    x = torch.randint(0, 97, (2, 32))
    y = torch.randint(0, 97, (2, 32))
    loss_ref = torch.nn.functional.cross_entropy(ref(x).flatten(0, 1), y.flatten())
    loss_ref.backward()
    xl, yl = shard_sequence(x, rank, world, layout), shard_sequence(y, rank, world, layout)
    loss = torch.nn.functional.cross_entropy(model(xl).flatten(0, 1), yl.flatten())
    loss.backward()
    lt = loss.detach().clone()
    dist.all_reduce(lt)
    tol = dict(rtol=1e-5, atol=1e-6)  # ring attention's tiles accumulate in fp32
    torch.testing.assert_close(lt / world, loss_ref.detach(), **tol)
    for (n, p), pr in zip(model.named_parameters(), ref.parameters()):
        g = p.grad.clone()
        dist.all_reduce(g)
        torch.testing.assert_close(g / world, pr.grad, msg=n, **tol)
    dist.destroy_process_group()


@pytest.mark.parametrize("layout", ["contiguous", "zigzag", "ulysses"])
def test_context_parallel_lm_matches_single_process(layout):
    spawn(_model_worker, 2, layout)
