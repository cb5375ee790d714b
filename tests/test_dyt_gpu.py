"""Weight gradients of the narrow projections (attention output, W2) from a transposed dY
(models/fused.py `_dy_transposed`, ops/gemm.py `mm_dyt_fp32`): same grads as the token-major path,
and every implementation `best` mode can pick (hipBLASLt default, autotuned hipBLASLt, cs336 GEMM)
matches an fp32 reference."""

import pytest
import torch

from cs336_systems import ops

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.mark.parametrize("mode", ["blas", "lt", "hip"])
@pytest.mark.parametrize("x_is_t", [False, True])
def test_mm_dyt_fp32_matches_reference(monkeypatch, mode, x_is_t):
    assert ops.load_ext(), ops.load_error()
    from cs336_systems.ops import gemm

    monkeypatch.setenv("CS336_GEMM", mode)
    torch.manual_seed(0)
    T, n_out, k_in = 1280, 320, 640
    dy = torch.randn(T, n_out, device=DEV).bfloat16()
    x = torch.randn(T, k_in, device=DEV).bfloat16()
    ref = dy.float().t() @ x.float()
    dyt = dy.t().contiguous()
    xo = x.t().contiguous() if x_is_t else x
    got = gemm.mm_dyt_fp32(dyt, xo, x_is_t)
    torch.testing.assert_close(got, ref, rtol=2e-3, atol=2e-3)
    out = torch.full((n_out, k_in), float("nan"), device=DEV)
    gemm.mm_dyt_fp32(dyt, xo, x_is_t, out=out)
    torch.testing.assert_close(out, ref, rtol=2e-3, atol=2e-3)


@pytest.mark.parametrize("ot", ["1", "0"])
def test_model_grads_with_and_without_dyt(monkeypatch, ot):
    from cs336_systems.models import BasicsTransformerLM

    monkeypatch.setenv("CS336_OT", ot)
    grads = []
    for flag in ("1", "0"):
        monkeypatch.setenv("CS336_DYT", flag)
        torch.manual_seed(0)
        m = BasicsTransformerLM(vocab_size=512, context_length=128, d_model=256, num_layers=2, num_heads=4, d_ff=512,
                                device=DEV)
        x = torch.randint(0, 512, (4, 128), device=DEV, generator=torch.Generator(DEV).manual_seed(1))
        with torch.autocast("cuda", dtype=torch.bfloat16):
            loss = ops.cross_entropy(m(x), x)
        loss.backward()
        grads.append({n: p.grad.clone() for n, p in m.named_parameters()})
    for n, g in grads[0].items():
        scale = g.abs().max().item() + 1e-12
        torch.testing.assert_close(g / scale, grads[1][n] / scale, rtol=0, atol=2e-3, msg=n)
