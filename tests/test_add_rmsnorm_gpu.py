"""Fused residual-add + RMSNorm kernels vs the fp32 PyTorch reference, and the model's chained
add+norm forward/backward vs the plain block loop."""

import pytest
import torch

from cs336_systems import ops
from cs336_systems.models import BasicsTransformerLM

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.mark.parametrize("H", [64, 1600, 2560, 3072])
@pytest.mark.parametrize("xdt,rdt", [(torch.float32, torch.bfloat16), (torch.float32, torch.float32), (torch.bfloat16, torch.bfloat16)])
@pytest.mark.parametrize("with_ds", [True, False])
def test_add_rmsnorm(H, xdt, rdt, with_ds):
    torch.manual_seed(0)
    M = 301
    x = torch.randn(M, H, device=DEV, dtype=xdt, requires_grad=True)
    r = torch.randn(M, H, device=DEV, dtype=rdt, requires_grad=True)
    w = (1 + 0.1 * torch.randn(H, device=DEV)).requires_grad_(True)
    s, y = ops.add_rmsnorm(x, r, w, 1e-5, torch.bfloat16)
    assert s.dtype == xdt and y.dtype == torch.bfloat16
    xr, rr, wr = (t.detach().double().requires_grad_(True) for t in (x, r, w))
    s_ref = xr + rr
    y_ref = wr * s_ref * torch.rsqrt(s_ref.pow(2).mean(-1, keepdim=True) + 1e-5)
    tol = 2e-2 if xdt == torch.bfloat16 else 1e-5
    torch.testing.assert_close(s.double(), s_ref, rtol=tol, atol=tol)
    torch.testing.assert_close(y.double(), y_ref, rtol=2e-2, atol=2e-2)
    dy = torch.randn(M, H, device=DEV, dtype=torch.bfloat16)
    ds = torch.randn(M, H, device=DEV, dtype=xdt) if with_ds else None
    if with_ds:
        torch.autograd.backward([s, y], [ds, dy])
        torch.autograd.backward([s_ref, y_ref], [ds.double(), dy.double()])
    else:
        y.backward(dy)
        y_ref.backward(dy.double())
    assert r.grad.dtype == rdt and x.grad.dtype == xdt
    gt = 5e-2 if (xdt == torch.bfloat16 or rdt == torch.bfloat16) else 1e-3
    torch.testing.assert_close(x.grad.double(), xr.grad, rtol=gt, atol=gt)
    torch.testing.assert_close(r.grad.double(), rr.grad, rtol=gt, atol=gt)
    torch.testing.assert_close(w.grad.double(), wr.grad, rtol=1e-2, atol=1e-2 * M**0.5)


def test_model_fused_residual_matches_block_loop(monkeypatch):
    torch.manual_seed(0)
    model = BasicsTransformerLM(vocab_size=512, context_length=64, d_model=256, num_layers=3, num_heads=4, d_ff=512, device=DEV)
    x = torch.randint(0, 512, (2, 64), device=DEV)
    y = torch.randint(0, 512, (2, 64), device=DEV)

    def run():
        model.zero_grad(set_to_none=True)
        with torch.autocast("cuda", dtype=torch.bfloat16):
            logits = model(x)
            loss = ops.cross_entropy(logits, y)
        loss.backward()
        return logits.float(), {n: p.grad.clone() for n, p in model.named_parameters()}

    assert model._fused_residual_ok(torch.empty(1, device=DEV))
    l_fused, g_fused = run()
    monkeypatch.setattr(BasicsTransformerLM, "_fused_residual_ok", lambda self, h: False)
    l_loop, g_loop = run()
    torch.testing.assert_close(l_fused, l_loop, rtol=2e-2, atol=2e-2)
    for n in g_loop:
        scale = g_loop[n].abs().max().item() + 1e-6
        torch.testing.assert_close(g_fused[n] / scale, g_loop[n] / scale, rtol=0, atol=3e-2, msg=n)


@pytest.mark.parametrize("H", [64, 1600, 2560])
@pytest.mark.parametrize("xdt", [torch.float32, torch.bfloat16])
def test_rmsnorm_bwd_add_t_matches_row_major(H, xdt):
    """The transposed-output residual backward (csrc/ops/rmsnorm.hip rmsnorm_bwd_add_t_kernel):
    dx, dw and the bf16 copy equal rmsnorm_bwd_add's bitwise, and dxT is that copy transposed."""
    assert ops.load_ext(), ops.load_error()
    torch.manual_seed(0)
    M = 16 * 37
    s = torch.randn(M, H, device=DEV, dtype=xdt)
    w = 1 + 0.1 * torch.randn(H, device=DEV)
    rstd = torch.rsqrt(s.float().pow(2).mean(-1) + 1e-5)
    dy = torch.randn(M, H, device=DEV, dtype=torch.bfloat16)
    ds = torch.randn(M, H, device=DEV, dtype=xdt)
    dx, dx2, dw = torch.ops.cs336.rmsnorm_bwd_add(dy, s, w, rstd, ds, True)
    tx, tx2, txt, tw = torch.ops.cs336.rmsnorm_bwd_add_t(dy, s, w, rstd, ds, True)
    assert torch.equal(dx, tx) and torch.equal(dx2, tx2)
    torch.testing.assert_close(tw, dw, rtol=1e-5, atol=1e-4)  # partial-row grouping differs
    assert txt.shape == (H, M) and torch.equal(txt, dx2.t())


def test_model_grads_fused_dyt_vs_transpose(monkeypatch):
    """Narrow-projection dW from the norm-written dYᵀ (offer/take) vs a separate transpose."""
    grads = []
    for flag in ("1", "0"):
        monkeypatch.setenv("CS336_DYT_FUSED", flag)
        from cs336_systems.models import fused

        fused._DYT_OFFERS.clear()
        torch.manual_seed(0)
        m = BasicsTransformerLM(vocab_size=512, context_length=128, d_model=256, num_layers=2, num_heads=4, d_ff=512,
                                device=DEV)
        x = torch.randint(0, 512, (4, 128), device=DEV, generator=torch.Generator(DEV).manual_seed(1))
        with torch.autocast("cuda", dtype=torch.bfloat16):
            loss = ops.cross_entropy(m(x), x)
        loss.backward()
        if flag == "1":
            assert not fused._DYT_OFFERS, "every offered dYᵀ should have been taken"
        grads.append({n: p.grad.clone() for n, p in m.named_parameters()})
    for n, g in grads[0].items():
        # projection grads are bitwise equal; the norm gains sum their partial rows in other groups
        torch.testing.assert_close(g, grads[1][n], rtol=1e-5, atol=1e-7, msg=n)
