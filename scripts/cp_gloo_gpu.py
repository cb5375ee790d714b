"""Context-parallel rehearsal on ONE GPU: 2 ranks share cuda:0 and pass K/V chunks over gloo
(GPU tensors staged through the host), running ring attention on the HIP FA2 kernels; each rank
checks its output and q/k/v gradients against single-call HIP attention on the full sequence.

    python scripts/cp_gloo_gpu.py [--layout zigzag|contiguous|ulysses]
"""

import argparse
import os
import sys

import torch
import torch.distributed as dist
import torch.multiprocessing as mp

sys.path.insert(0, __file__.rsplit("/scripts/", 1)[0])


def worker(rank, world, layout, port):
    from cs336_systems.ops.flash_attention import FlashAttentionHIP
    from cs336_systems.parallel import ring_attention, shard_sequence, ulysses_attention

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.manual_seed(0)
    B, H, N, D = 2, 4, 1024, 64
    q, k, v, do = (torch.randn(B, H, N, D, device="cuda", dtype=torch.bfloat16) for _ in range(4))
    qf, kf, vf = (t.clone().requires_grad_(True) for t in (q, k, v))
    FlashAttentionHIP.apply(qf, kf, vf, True).backward(do)
    of = FlashAttentionHIP.apply(qf.detach(), kf.detach(), vf.detach(), True)
    sh = lambda t: shard_sequence(t, rank, world, layout, dim=2)  # noqa: E731
    ql, kl, vl = (sh(t).requires_grad_(True) for t in (q, k, v))
    o = ulysses_attention(ql, kl, vl, None, True) if layout == "ulysses" else ring_attention(ql, kl, vl, None, True, layout)
    o.backward(sh(do))
    torch.testing.assert_close(o.float(), sh(of).float(), rtol=2e-2, atol=2e-2)
    for got, ref in ((ql, qf), (kl, kf), (vl, vf)):
        torch.testing.assert_close(got.grad.float(), sh(ref.grad).float(), rtol=5e-2, atol=5e-2)
    torch.cuda.synchronize()
    print(f"rank {rank}: context-parallel attention ({layout}, world {world}) matches full HIP FA2", flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--layout", default="zigzag")
    ap.add_argument("--world", type=int, default=2)
    a = ap.parse_args()
    from cs336_systems.parallel.comm import find_free_port

    mp.spawn(worker, args=(a.world, a.layout, find_free_port()), nprocs=a.world, join=True)
