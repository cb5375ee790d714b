"""ZeRO-2 data parallelism with the sharded fused AdamW (parallel/zero.py) on CPU/gloo: each rank
trains on its slice of the batch, gradients are reduce-scattered, every rank updates only its
shards and the parameters are all-gathered before the next forward — and after every step the
parameters equal single-process training on the whole batch with the same AdamW. Covers frozen and
tied parameters, one-bucket / per-parameter / small buckets, 2 and 4 ranks, global-norm clipping
and a Transformer LM."""

import os

import pytest
import torch
import torch.distributed as dist
import torch.nn.functional as F

from cs336_systems.models import BasicsTransformerLM
from cs336_systems.ops import FusedAdamW, clip_grad_norm_
from cs336_systems.parallel.zero import ZeroDDP

from .common import FIXTURES_PATH, ToyModel, ToyModelWithTiedWeights, spawn

OPT = dict(lr=0.05, betas=(0.9, 0.999), eps=1e-8, weight_decay=0.1)


def _init(rank, world):
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world))
    dist.init_process_group("gloo", rank=rank, world_size=world)


def _toy_worker(rank, world, model_cls, bucket_mb):
    _init(rank, world)
    torch.manual_seed(rank)  # different inits: the wrapper must broadcast rank 0's
    base = model_cls()
    torch.manual_seed(0)
    ref = model_cls()
    ref.load_state_dict(base.state_dict())
    dist.broadcast_object_list(obj := [ref.state_dict()], src=0)
    ref.load_state_dict(obj[0])
    zero = ZeroDDP(base, bucket_size_mb=bucket_mb, **OPT)
    for a, b in zip(zero.module.state_dict().values(), ref.state_dict().values()):
        assert torch.equal(a, b)
    ref_opt = FusedAdamW([p for p in ref.parameters() if p.requires_grad], **OPT)
    opt = zero.optimizer
    x_all = torch.load(FIXTURES_PATH / "ddp_test_data.pt", weights_only=True)
    y_all = torch.load(FIXTURES_PATH / "ddp_test_labels.pt", weights_only=True)
    per = x_all.shape[0] // world
    for it in range(5):
        g = torch.Generator().manual_seed(42 + it)
        perm = torch.randperm(x_all.shape[0], generator=g)
        x_all, y_all = x_all[perm], y_all[perm]
        ref_opt.zero_grad(set_to_none=True)
        F.mse_loss(ref(x_all), y_all).backward()
        ref_opt.step()
        opt.zero_grad(set_to_none=True)
        xs, ys = x_all[rank * per : (rank + 1) * per], y_all[rank * per : (rank + 1) * per]
        F.mse_loss(zero(xs), ys).backward()
        zero.finish_gradient_synchronization()
        opt.step()
        sd = zero.state_dict()
        for (n, a), b in zip(sd.items(), ref.state_dict().values()):
            torch.testing.assert_close(a, b, rtol=1e-5, atol=1e-6, msg=lambda m, n=n, it=it: f"iter {it} {n}: {m}")
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("model_cls", [ToyModel, ToyModelWithTiedWeights])
@pytest.mark.parametrize("bucket_mb", [None, 0.0001, 0.002])
def test_zero_matches_single_process_toy(model_cls, bucket_mb):
    spawn(_toy_worker, 2, model_cls, bucket_mb)


def _lm_worker(rank, world, clip):
    _init(rank, world)
    cfg = dict(vocab_size=64, context_length=16, d_model=32, num_layers=2, num_heads=2, d_ff=64)
    torch.manual_seed(0)
    ref = BasicsTransformerLM(**cfg)
    torch.manual_seed(0)
    model = BasicsTransformerLM(**cfg)
    zero = ZeroDDP(model, bucket_size_mb=0.02, **OPT)
    assert len(zero.buckets) > 1
    ref_opt = FusedAdamW(ref.parameters(), **OPT)
    opt = zero.optimizer
    B = 2 * world
    for it in range(3):
        g = torch.Generator().manual_seed(it)
        x = torch.randint(0, 64, (B, 16), generator=g)
        ref_opt.zero_grad(set_to_none=True)
        F.cross_entropy(ref(x).reshape(-1, 64), x.reshape(-1)).backward()
        if clip:
            n_ref = clip_grad_norm_(ref.parameters(), clip)
        ref_opt.step()
        opt.zero_grad(set_to_none=True)
        xs = x[rank * 2 : (rank + 1) * 2]
        F.cross_entropy(zero(xs).reshape(-1, 64), xs.reshape(-1)).backward()
        zero.finish_gradient_synchronization()
        if clip:
            n = zero.clip_grad_norm_(clip)
            torch.testing.assert_close(n.float(), n_ref.float(), rtol=1e-5, atol=1e-6)
        opt.step()
        # Adam's early steps are ~lr·sign(g): a gradient within rounding of zero (the two ranks sum
        # it in a different order than the single process) moves its weight by up to ~1e-4
        for (name, a), b in zip(zero.state_dict().items(), ref.state_dict().values()):
            torch.testing.assert_close(a, b, rtol=1e-4, atol=1e-4, msg=lambda m, n=name, it=it: f"iter {it} {n}: {m}")
    for t in zero.state_dict().values():  # every rank holds identical parameters
        got = [torch.empty_like(t) for _ in range(world)]
        dist.all_gather(got, t)
        assert all(torch.equal(g_, t) for g_ in got)
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world,clip", [(1, 0.0), (2, 0.0), (4, 0.0), (2, 0.05)])
def test_zero_lm_matches_single_process(world, clip):
    spawn(_lm_worker, world, clip)
