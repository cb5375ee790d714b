"""Tensor parallelism on the GPU path: 2 ranks share cuda:0 (gloo, host-staged all-reduces), each
holding half the heads and half of d_ff of a fused-layout LM under bf16 autocast — the grouped QKV /
W1|W3 GEMMs, HIP RoPE + FA2 and the fused residual/RMSNorm loop all run on the shards — and the
logits, loss and gathered gradients match the single-process model."""

import os

import pytest
import torch
import torch.distributed as dist

pytestmark = pytest.mark.gpu

CFG = dict(vocab_size=512, context_length=128, d_model=256, num_layers=2, num_heads=4, d_ff=1024)


def _worker(rank, world, port):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from cs336_systems import ops
    from cs336_systems.models import BasicsTransformerLM
    from cs336_systems.parallel.tensor_parallel import _tp_split, tensor_parallel_

    torch.manual_seed(0)
    ref = BasicsTransformerLM(**CFG, device="cuda", fused_layout=True)
    torch.manual_seed(0)
    model = BasicsTransformerLM(**CFG, device="cuda", fused_layout=True)
    tensor_parallel_(model)
    x = torch.randint(0, 512, (2, 128), device="cuda", generator=torch.Generator("cuda").manual_seed(1))
    outs = []
    for m in (ref, model):
        with torch.autocast("cuda", dtype=torch.bfloat16):
            logits = m(x)
            loss = ops.cross_entropy(logits, x)
        loss.backward()
        outs.append((logits.float(), loss.float()))
    torch.testing.assert_close(outs[1][0], outs[0][0], rtol=3e-2, atol=3e-2)
    torch.testing.assert_close(outs[1][1], outs[0][1], rtol=1e-2, atol=1e-2)
    named_ref = dict(ref.named_parameters())
    for n, p in model.named_parameters():
        g = named_ref[n].grad
        dim = _tp_split(n)
        if dim is not None:
            k = g.shape[dim] // world
            g = g.narrow(dim, rank * k, k)
        scale = g.abs().max().item() + 1e-6
        torch.testing.assert_close(p.grad / scale, g / scale, rtol=0, atol=3e-2, msg=n)
    print(f"rank {rank}: tensor-parallel step matches", flush=True)
    dist.destroy_process_group()


def test_tensor_parallel_two_ranks_one_gpu():
    import torch.multiprocessing as mp

    from cs336_systems.parallel.comm import find_free_port

    mp.spawn(_worker, args=(2, find_free_port()), nprocs=2, join=True)
