"""Tensor parallelism (parallel/tensor_parallel.py) on CPU/gloo: a TP-sharded LM (heads and d_ff
split over 2 or 4 ranks) gives the single-process logits, loss and gradients (sharded weights'
gradients equal the matching slices of the full gradients, replicated ones are equal), the
gathered state dict equals the full model's, and AdamW steps on the shards keep it that way."""

import os

import pytest
import torch
import torch.distributed as dist
import torch.nn.functional as F

from cs336_systems.models import BasicsTransformerLM
from cs336_systems.ops import FusedAdamW
from cs336_systems.parallel.tensor_parallel import _tp_split, gather_tp_state_dict, tensor_parallel_

from .common import spawn

CFG = dict(vocab_size=97, context_length=32, d_model=64, num_layers=2, num_heads=4, d_ff=96)
OPT = dict(lr=1e-3, betas=(0.9, 0.95), eps=1e-8, weight_decay=0.01)


def _worker(rank, world):
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.manual_seed(0)
    ref = BasicsTransformerLM(**CFG).double()
    model = BasicsTransformerLM(**CFG).double()
    model.load_state_dict(ref.state_dict())
    tensor_parallel_(model)
    assert model.layers[0].attn.num_heads == 4 // world
    ref_opt, opt = FusedAdamW(ref.parameters(), **OPT), FusedAdamW(model.parameters(), **OPT)
    tol = dict(rtol=1e-9, atol=1e-10)
    for it in range(2):
        x = torch.randint(0, 97, (2, 32), generator=torch.Generator().manual_seed(it))
        for m, o in ((ref, ref_opt), (model, opt)):
            o.zero_grad(set_to_none=True)
        logits_ref = ref(x)
        logits = model(x)
        torch.testing.assert_close(logits, logits_ref, **tol)
        F.cross_entropy(logits_ref.flatten(0, 1), x.flatten()).backward()
        F.cross_entropy(logits.flatten(0, 1), x.flatten()).backward()
        named_ref = dict(ref.named_parameters())
        for n, p in model.named_parameters():
            g = named_ref[n].grad
            dim = _tp_split(n)
            if dim is not None:
                k = g.shape[dim] // world
                g = g.narrow(dim, rank * k, k)
            torch.testing.assert_close(p.grad, g, msg=n, **tol)
        ref_opt.step()
        opt.step()
    full = gather_tp_state_dict(model)
    for n, t in ref.state_dict().items():
        torch.testing.assert_close(full[n], t, msg=n, **tol)
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 4])
def test_tensor_parallel_matches_single_process(world):
    spawn(_worker, world)


def _reject_worker(rank, world):
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    with pytest.raises(ValueError):
        tensor_parallel_(BasicsTransformerLM(**dict(CFG, d_model=48, num_heads=3)))
    with pytest.raises(ValueError):
        tensor_parallel_(torch.nn.Linear(4, 4))
    dist.destroy_process_group()


def test_tensor_parallel_rejects_indivisible_heads():
    spawn(_reject_worker, 2)
