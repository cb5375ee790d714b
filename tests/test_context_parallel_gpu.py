"""Ring attention on the HIP FA2 kernels (parallel/context_parallel.py), world 1 over RCCL: with the
zigzag layout one rank holds two sub-chunks, so the second attends the first (full) and itself
(causal) and the partials are merged by their LSE — compared with the single-call HIP FA2 and an
fp32 reference, forward and backward; and a context-parallel LM step against the plain model."""

import os

import pytest
import torch
import torch.distributed as dist

from cs336_systems import ops
from cs336_systems.models import BasicsTransformerLM
from cs336_systems.ops.flash_attention import FlashAttentionHIP, naive_attention
from cs336_systems.parallel import disable_context_parallel, enable_context_parallel, ring_attention, ulysses_attention
from cs336_systems.parallel.comm import find_free_port

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.fixture(scope="module", autouse=True)
def rccl_world1():
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(find_free_port()))
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device(DEV, 0))
    yield
    dist.destroy_process_group()


@pytest.mark.parametrize("D", [64, 128])
def test_ring_attention_hip_zigzag_world1(D):
    torch.manual_seed(0)
    B, H, N = 2, 4, 512
    q, k, v, do = (torch.randn(B, H, N, D, device=DEV, dtype=torch.bfloat16) for _ in range(4))
    ref = [t.float().requires_grad_(True) for t in (q, k, v)]
    naive_attention(*ref, is_causal=True).backward(do.float())
    ql, kl, vl = (t.clone().requires_grad_(True) for t in (q, k, v))
    o = ring_attention(ql, kl, vl, None, True, "zigzag")
    o.backward(do)
    qf, kf, vf = (t.clone().requires_grad_(True) for t in (q, k, v))
    of = FlashAttentionHIP.apply(qf, kf, vf, True)
    of.backward(do)
    with torch.no_grad():
        o_ref = naive_attention(*[t.detach() for t in ref], is_causal=True)
    torch.testing.assert_close(o.float(), o_ref, rtol=2e-2, atol=2e-2)
    torch.testing.assert_close(o.float(), of.float(), rtol=2e-2, atol=2e-2)
    for got, r in zip((ql, kl, vl), ref):
        torch.testing.assert_close(got.grad.float(), r.grad, rtol=5e-2, atol=5e-2)


def test_ulysses_world1_matches_hip_fa():
    """World 1 over RCCL: the all-to-alls are identities, the attention is one HIP FA2 call."""
    torch.manual_seed(1)
    q, k, v, do = (torch.randn(2, 4, 512, 64, device=DEV, dtype=torch.bfloat16) for _ in range(4))
    ql, kl, vl = (t.clone().requires_grad_(True) for t in (q, k, v))
    o = ulysses_attention(ql, kl, vl, None, True)
    o.backward(do)
    qf, kf, vf = (t.clone().requires_grad_(True) for t in (q, k, v))
    of = FlashAttentionHIP.apply(qf, kf, vf, True)
    of.backward(do)
    torch.testing.assert_close(o, of, rtol=0, atol=0)
    for a, b in ((ql, qf), (kl, kf), (vl, vf)):
        torch.testing.assert_close(a.grad, b.grad, rtol=0, atol=0)


def test_context_parallel_lm_world1_matches_plain():
    torch.manual_seed(0)
    model = BasicsTransformerLM(vocab_size=512, context_length=256, d_model=256, num_layers=2, num_heads=4, d_ff=512, device=DEV)
    x = torch.randint(0, 512, (2, 256), device=DEV)

    def run():
        model.zero_grad(set_to_none=True)
        with torch.autocast("cuda", dtype=torch.bfloat16):
            loss = ops.cross_entropy(model(x), x)
        loss.backward()
        return loss.detach().float(), {n: p.grad.float().clone() for n, p in model.named_parameters()}

    loss_ref, g_ref = run()
    enable_context_parallel(model, None, "zigzag")
    loss_cp, g_cp = run()
    disable_context_parallel(model)
    torch.testing.assert_close(loss_cp, loss_ref, rtol=1e-2, atol=1e-2)
    for n in g_ref:
        torch.testing.assert_close(g_cp[n], g_ref[n], rtol=5e-2, atol=5e-3, msg=n)


@pytest.mark.parametrize("world,layout", [(2, "zigzag"), (4, "contiguous"), (4, "zigzag"), (2, "ulysses"), (4, "ulysses")])
def test_ring_attention_multirank_one_gpu(world, layout):
    """2-4 ranks share cuda:0 (gloo, host-staged P2P): the multi-hop ring on the HIP kernels."""
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    r = subprocess.run([sys.executable, os.path.join(root, "scripts", "cp_gloo_gpu.py"), "--layout", layout, "--world", str(world)],
                       capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    assert r.stdout.count("matches full HIP FA2") == world
