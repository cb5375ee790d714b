"""ZeRO-1 with bf16 weight shadows on GPU tensors: 2 ranks sharing cuda:0 over gloo. After every
step each replica's shadows equal bf16(master) — including the all-gathered parameters this rank
does not own — and the replicas track a single-process FusedAdamW run."""

import copy

import pytest
import torch
import torch.distributed as dist

from .common import spawn

pytestmark = pytest.mark.gpu


def _worker(rank, world):
    from cs336_systems import ops
    from cs336_systems.models import BasicsTransformerLM
    from cs336_systems.models.fused import get_shadow, shadow_valid
    from cs336_systems.parallel import ShardedOptimizer

    dist.init_process_group("gloo", rank=rank, world_size=world)
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    torch.manual_seed(0)
    model = BasicsTransformerLM(vocab_size=256, context_length=32, d_model=64, num_layers=2, num_heads=2, d_ff=128, device=dev)
    ref = copy.deepcopy(model)
    okw = dict(lr=1e-3, betas=(0.9, 0.95), eps=1e-8, weight_decay=0.01)
    opt = ShardedOptimizer(model.parameters(), ops.FusedAdamW, bf16_shadows=True, **okw)
    ref_opt = ops.FusedAdamW(ref.parameters(), **okw)
    g = torch.Generator(device=dev).manual_seed(1)
    for _ in range(3):
        x = torch.randint(0, 256, (2, 32), device=dev, generator=g)
        for m, o in ((model, opt), (ref, ref_opt)):
            o.zero_grad(set_to_none=True)
            with torch.autocast("cuda", dtype=torch.bfloat16):
                loss = ops.cross_entropy(m(x), x)
            loss.backward()
            o.step()
        for p in model.parameters():
            if p.dim() == 2:
                assert shadow_valid(p), "shadow not marked synced"
                torch.testing.assert_close(get_shadow(p), p.detach().bfloat16(), rtol=0, atol=0)
    # the GPU embedding backward accumulates with atomics, so the two ranks' gradients (and the
    # reference's) can differ in the last bits; Adam normalizes updates to ~lr, so a near-zero
    # gradient entry can move by up to ~2·lr per step between runs
    for p, q in zip(model.parameters(), ref.parameters()):
        torch.testing.assert_close(p, q, rtol=0, atol=2 * okw["lr"] * 3 + 1e-5)
    dist.barrier()
    dist.destroy_process_group()


def test_zero1_shadows_two_ranks_one_gpu():
    spawn(_worker, 2)
