"""RMSNorm backward variants that write the weight gradient into a caller's buffer (a DDP bucket
view: ops/rmsnorm.py ``_dw_target``) give the same bits as the allocating ops, and a DDP-wrapped
model adopts those views as ``.grad`` without a copy."""

import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _inputs(M=512, H=1600, dt=torch.float32):
    torch.manual_seed(0)
    x = torch.randn(M, H, device=DEV, dtype=dt)
    dy = torch.randn(M, H, device=DEV, dtype=torch.bfloat16)
    w = torch.rand(H, device=DEV) + 0.5
    rstd = torch.rsqrt(x.float().pow(2).mean(-1) + 1e-5)
    dres = torch.randn(M, H, device=DEV, dtype=dt)
    return dy, x, w, rstd, dres


def test_rmsnorm_bwd_into_bitwise():
    dy, x, w, rstd, _ = _inputs()
    cs = torch.ops.cs336
    dx, dw = cs.rmsnorm_bwd(dy, x, w, rstd)
    out = torch.full_like(dw, float("nan"))
    dx2 = cs.rmsnorm_bwd_into(dy, x, w, rstd, out)
    assert torch.equal(dx, dx2) and torch.equal(dw, out)


@pytest.mark.parametrize("emit", [False, True])
def test_rmsnorm_bwd_add_into_bitwise(emit):
    dy, x, w, rstd, dres = _inputs()
    cs = torch.ops.cs336
    dx, dxb, dw = cs.rmsnorm_bwd_add(dy, x, w, rstd, dres, emit)
    out = torch.full_like(dw, float("nan"))
    dx2, dxb2 = cs.rmsnorm_bwd_add_into(dy, x, w, rstd, dres, emit, out)
    assert torch.equal(dx, dx2) and torch.equal(dw, out)
    if emit:
        assert torch.equal(dxb, dxb2)
    dx, dxb, dxt, dw = cs.rmsnorm_bwd_add_t(dy, x, w, rstd, dres, True)
    out = torch.full_like(dw, float("nan"))
    dx2, dxb2, dxt2 = cs.rmsnorm_bwd_add_t_into(dy, x, w, rstd, dres, True, out)
    assert torch.equal(dx, dx2) and torch.equal(dxb, dxb2) and torch.equal(dxt, dxt2) and torch.equal(dw, out)


def test_ddp_world1_grads_land_in_bucket_views():
    """Norm weights and the embedding table get their gradients written into the bucket views (the
    .grad tensors alias the buckets) and the step equals the unwrapped one."""
    import os

    import torch.distributed as dist

    from cs336_systems import ops
    from cs336_systems.models import BasicsTransformerLM
    from cs336_systems.parallel import DDPBucketed
    from cs336_systems.parallel.comm import find_free_port

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(find_free_port()))
    dist.init_process_group("nccl", rank=0, world_size=1)
    try:
        def make():
            torch.manual_seed(0)
            return BasicsTransformerLM(vocab_size=512, context_length=64, d_model=256, num_layers=2, num_heads=4,
                                       d_ff=768, device=DEV)

        ref, m = make(), make()
        ddp = DDPBucketed(m, bucket_size_mb=1)
        x = torch.randint(0, 512, (4, 64), device=DEV)
        for model in (ref, ddp):
            for p in model.parameters():
                p.grad = None
            with torch.autocast("cuda", dtype=torch.bfloat16):
                ops.cross_entropy(model(x), x).backward()
        ddp.finish_gradient_synchronization()
        for (n, p), q in zip(m.named_parameters(), ref.parameters()):
            view = ddp._views[p]
            assert p.grad.data_ptr() == view.data_ptr(), n
            torch.testing.assert_close(p.grad, q.grad, rtol=0, atol=0, msg=n)
    finally:
        dist.destroy_process_group()
