"""RoPE in the QKV GEMM's store (gemm8 epi 3, models/fused.py QKVRopeLinearFn): the kernel against
gemm8 + the separate RoPE kernel and an fp32 PyTorch reference of the same op, and the attention
module with the fused store against the unfused path (forward and every gradient)."""

import pytest
import torch

pytestmark = pytest.mark.gpu


def _cs():
    from cs336_systems import ops

    if not torch.cuda.is_available():
        pytest.skip("needs a GPU")
    assert ops.load_ext(), ops.load_error()
    return torch.ops.cs336


def _rand(*s, scale=1.0, seed=0):
    g = torch.Generator(device="cuda").manual_seed(seed)
    return ((torch.rand(*s, device="cuda", generator=g) * 2 - 1) * scale).to(torch.bfloat16)


def _tables(ctx, dk, theta=10000.0):
    inv = 1.0 / (theta ** (torch.arange(0, dk, 2, device="cuda", dtype=torch.float64) / dk))
    ang = torch.arange(ctx, device="cuda", dtype=torch.float64)[:, None] * inv[None, :]
    return torch.cos(ang).float().contiguous(), torch.sin(ang).float().contiguous()


def _rope_ref(y, cos, sin, pos, rope_cols, dk):
    """fp32 interleaved-pair rotation of the columns < rope_cols of y (M, N); pos (M,) int64."""
    y = y.float().clone()
    M = y.shape[0]
    qk = y[:, :rope_cols].view(M, -1, dk // 2, 2)
    c, s = cos[pos][:, None, :], sin[pos][:, None, :]
    x0, x1 = qk[..., 0].clone(), qk[..., 1].clone()
    qk[..., 0] = c * x0 - s * x1
    qk[..., 1] = s * x0 + c * x1
    return y


@pytest.mark.parametrize("B,N,H,dk,K", [(2, 128, 5, 64, 320), (1, 512, 25, 64, 1600), (4, 64, 4, 80, 320),
                                        (2, 256, 4, 128, 512)])
@pytest.mark.parametrize("given_pos", [False, True])
def test_gemm8_rope_kernel(B, N, H, dk, K, given_pos):
    cs = _cs()
    M, Nout = B * N, 3 * H * dk
    if not cs.gemm8_ok(M, Nout, K, 3, 2 * H * dk) or dk > 96:
        pytest.skip("gemm8 epi 3 does not take this shape")
    x, w = _rand(M, K, seed=1), _rand(Nout, K, scale=0.1, seed=2)
    cos, sin = _tables(max(N, 600), dk)
    if given_pos:
        pos = torch.randint(0, cos.shape[0], (M,), device="cuda", dtype=torch.int64)
    else:
        pos = torch.arange(N, device="cuda", dtype=torch.int64).repeat(B)
    out = torch.empty(M, Nout, device="cuda", dtype=torch.bfloat16)
    cs.gemm8_rope(x, w, out, cos, sin, pos if given_pos else None, N, 2 * H * dk, dk)
    # fp32 reference of the op
    ref = _rope_ref(x.float() @ w.float().t(), cos, sin, pos, 2 * H * dk, dk)
    rel = float((out.float() - ref).norm() / ref.norm())
    assert rel < 5e-3, rel
    # the unfused pair: gemm8 then the RoPE kernel on the q|k heads (same rounding points)
    plain = torch.empty_like(out)
    cs.gemm8(x, w, plain, 0, 0, None, None, 0)
    qk = plain.view(B, N, 3 * H, dk)[:, :, : 2 * H].transpose(1, 2)
    cs.rope_into(qk, cos, sin, pos.view(B, N) if given_pos else None, False, qk)
    diff = (out.float() - plain.float()).abs()
    assert float(diff.max()) <= 2 * float(ref.abs().max()) * 2 ** -8  # at most a bf16 ulp apart
    assert float((diff > 0).float().mean()) < 0.02
    # v columns untouched by the rotation
    torch.testing.assert_close(out[:, 2 * H * dk:], plain[:, 2 * H * dk:], rtol=0, atol=0)


def _attn_run(m, x, dy, monkeypatch, fused: bool):
    monkeypatch.setenv("CS336_QKV_ROPE", "1" if fused else "0")
    monkeypatch.setenv("CS336_GEMM", "best")
    for p in m.parameters():
        p.grad = None
    xx = x.clone().requires_grad_(True)
    with torch.autocast("cuda", dtype=torch.bfloat16):
        out = m(xx)
    out.backward(dy)
    return [out.float()] + [xx.grad.float()] + [p.grad.float().clone() for p in m.parameters()]


@pytest.mark.parametrize("d_model,H,N", [(1600, 25, 512), (320, 5, 256)])
def test_attention_with_rope_in_gemm(monkeypatch, d_model, H, N):
    from cs336_systems.models.fused import attach_bf16_shadows
    from cs336_systems.models.transformer import CausalMultiHeadSelfAttention, RotaryEmbedding

    _cs()
    torch.manual_seed(0)
    rope = RotaryEmbedding(N, d_model // H, 10000.0, "cuda")
    m = CausalMultiHeadSelfAttention(d_model, H, rope, device="cuda")
    m.group_()
    attach_bf16_shadows(m)
    x = torch.randn(2, N, d_model, device="cuda")
    dy = torch.randn(2, N, d_model, device="cuda")
    got = _attn_run(m, x, dy, monkeypatch, True)
    ref = _attn_run(m, x, dy, monkeypatch, False)
    for g, r in zip(got, ref):
        rel = float((g - r).norm() / r.norm().clamp_min(1e-30))
        assert rel < 1e-2, rel
