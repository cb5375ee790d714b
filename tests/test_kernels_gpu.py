"""Numerics of every HIP kernel against a plain PyTorch fp32 reference of the same op (GPU only).

Also asserts that the native extension is actually loaded on the GPU box (no silent eager
fallback: the ops raise if the .so is missing)."""

import math

import pytest
import torch

from cs336_systems import ops
from cs336_systems.ops import _ext

pytestmark = pytest.mark.gpu

DEV = "cuda"


def test_extension_loaded():
    assert _ext.load_ext(), _ext.load_error()
    assert hasattr(torch.ops.cs336, "fa_fwd")


# ---------------------------------------------------------------------------------- RMSNorm
@pytest.mark.parametrize("H", [64, 1600, 2560, 3072, 4100])
@pytest.mark.parametrize("xdt,odt", [(torch.float32, torch.float32), (torch.float32, torch.bfloat16), (torch.bfloat16, torch.bfloat16)])
def test_rmsnorm(H, xdt, odt):
    torch.manual_seed(0)
    x = torch.randn(37, H, device=DEV, dtype=xdt, requires_grad=True)
    w = (1 + 0.1 * torch.randn(H, device=DEV)).requires_grad_(True)
    y = ops.rmsnorm(x, w, 1e-5, out_dtype=odt)
    xr = x.detach().float().requires_grad_(True)
    wr = w.detach().clone().requires_grad_(True)
    yr = ops.rmsnorm_ref(xr, wr, 1e-5)
    tol = 2e-2 if odt == torch.bfloat16 or xdt == torch.bfloat16 else 1e-5
    torch.testing.assert_close(y.float(), yr, rtol=tol, atol=tol)
    g = torch.randn_like(yr)
    y.backward(g.to(y.dtype))
    yr.backward(g.to(y.dtype).float())
    torch.testing.assert_close(x.grad.float(), xr.grad, rtol=tol * 2, atol=tol * 2)
    torch.testing.assert_close(w.grad, wr.grad, rtol=5e-2 if tol > 1e-4 else 1e-4, atol=tol * 10)


# ---------------------------------------------------------------------------------- RoPE
@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("with_pos", [False, True])
@pytest.mark.parametrize("D", [32, 64, 80, 128])
def test_rope(dt, with_pos, D):
    torch.manual_seed(0)
    B, N, H, ctx = 2, 33, 3, 64
    from cs336_systems.ops.rope import _hip_layout_ok

    assert _hip_layout_ok(torch.empty(B, N, H, D, device=DEV, dtype=dt).transpose(1, 2))
    from cs336_systems.models import RotaryEmbedding

    re = RotaryEmbedding(ctx, D, 10000.0).to(DEV)
    xb = torch.randn(B, N, H, D, device=DEV, dtype=dt)
    x = xb.transpose(1, 2).requires_grad_(False)  # (B,H,N,D) strided view
    pos = torch.randint(0, ctx, (B, N), device=DEV) if with_pos else None
    xg = x.detach().clone().requires_grad_(True)
    y = ops.rope(xg, re.cos, re.sin, pos)
    p = pos[:, None, :] if with_pos else torch.arange(N, device=DEV)
    yr = ops.rope_ref(x.float(), re.cos, re.sin, p)
    tol = 1e-5 if dt == torch.float32 else 1e-2
    torch.testing.assert_close(y.float(), yr, rtol=tol, atol=tol)
    assert y.transpose(1, 2).is_contiguous()  # (B,N,H,D) memory order
    g = torch.randn_like(yr)
    y.backward(g.to(dt))
    # R is orthogonal: backward = inverse rotation of g
    xr = x.float().clone().requires_grad_(True)
    ops.rope_ref(xr, re.cos, re.sin, p).backward(g.to(dt).float())
    torch.testing.assert_close(xg.grad.float(), xr.grad, rtol=tol * 2, atol=tol * 2)


# ---------------------------------------------------------------------------------- SwiGLU
@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("n", [4096, 1001])
def test_silu_mul(dt, n):
    torch.manual_seed(0)
    a = torch.randn(3, n, device=DEV, dtype=dt, requires_grad=True)
    b = torch.randn(3, n, device=DEV, dtype=dt, requires_grad=True)
    h = ops.silu_mul(a, b)
    ar, br = a.detach().float().requires_grad_(True), b.detach().float().requires_grad_(True)
    hr = ops.silu_mul_ref(ar, br)
    tol = 1e-5 if dt == torch.float32 else 2e-2
    torch.testing.assert_close(h.float(), hr, rtol=tol, atol=tol)
    g = torch.randn_like(hr)
    h.backward(g.to(dt))
    hr.backward(g.to(dt).float())
    torch.testing.assert_close(a.grad.float(), ar.grad, rtol=tol * 2, atol=tol * 2)
    torch.testing.assert_close(b.grad.float(), br.grad, rtol=tol * 2, atol=tol * 2)


# ---------------------------------------------------------------------------------- cross entropy
@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("V", [10000, 1003])
def test_cross_entropy(dt, V):
    torch.manual_seed(0)
    z = (3 * torch.randn(2, 65, V, device=DEV)).to(dt).requires_grad_(True)
    t = torch.randint(0, V, (2, 65), device=DEV)
    loss = ops.cross_entropy(z, t)
    zr = z.detach().float().requires_grad_(True)
    lr = torch.nn.functional.cross_entropy(zr.view(-1, V), t.view(-1))
    torch.testing.assert_close(loss, lr, rtol=1e-4, atol=1e-4)
    (2.0 * loss).backward()
    (2.0 * lr).backward()
    tol = 1e-6 if dt == torch.float32 else 1e-4
    torch.testing.assert_close(z.grad.float(), zr.grad, rtol=1e-2, atol=tol)


# ---------------------------------------------------------------------------------- AdamW / clip
def test_fused_adamw_matches_reference():
    from cs336_basics.optimizer import ReferenceAdamW

    torch.manual_seed(0)
    shapes = [(1600, 1600), (7,), (33, 5), (100003,), (10000, 16)]
    ps = [torch.randn(s, device=DEV) for s in shapes]
    p1 = [torch.nn.Parameter(p.clone()) for p in ps]
    p2 = [torch.nn.Parameter(p.clone()) for p in ps]
    o1 = ops.FusedAdamW(p1, lr=1e-3, betas=(0.9, 0.95), eps=1e-8, weight_decay=0.1)
    o2 = ReferenceAdamW(p2, lr=1e-3, betas=(0.9, 0.95), eps=1e-8, weight_decay=0.1)
    for _ in range(5):
        for a, b in zip(p1, p2):
            g = torch.randn_like(a)
            a.grad, b.grad = g.clone(), g.clone()
        o1.step()
        o2.step()
    for a, b in zip(p1, p2):
        torch.testing.assert_close(a, b, rtol=1e-6, atol=1e-7)
    for a, b in zip(p1, p2):
        torch.testing.assert_close(o1.state[a]["m"], o2.state[b]["m"], rtol=1e-6, atol=1e-8)


def test_clip_grad_norm():
    torch.manual_seed(0)
    ps = [torch.nn.Parameter(torch.randn(s, device=DEV)) for s in [(1000, 3), (5,), (70001,)]]
    for p in ps:
        p.grad = torch.randn_like(p)
    ref = [p.grad.clone() for p in ps]
    n = torch.sqrt(sum((g.double() ** 2).sum() for g in ref)).float()
    out = ops.clip_grad_norm_(ps, 1.0)
    torch.testing.assert_close(out, n, rtol=1e-5, atol=1e-5)
    c = min(1.0, 1.0 / (n.item() + 1e-6))
    for p, g in zip(ps, ref):
        torch.testing.assert_close(p.grad, g * c, rtol=1e-5, atol=1e-6)


# ---------------------------------------------------------------------------------- FlashAttention
def _ref_attn(q, k, v, causal):
    d = q.shape[-1]
    s = torch.matmul(q.double(), k.double().transpose(-1, -2)) / math.sqrt(d)
    if causal:
        n, m = q.shape[-2], k.shape[-2]
        mask = torch.arange(n, device=q.device)[:, None] >= torch.arange(m, device=q.device)[None, :]
        s = s.masked_fill(~mask, float("-inf"))
    L = torch.logsumexp(s, -1)
    o = torch.matmul(torch.softmax(s, -1), v.double())
    return o, L


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16, torch.float16])
@pytest.mark.parametrize("D", [32, 64, 128])
@pytest.mark.parametrize("causal", [False, True])
@pytest.mark.parametrize("N", [128, 200, 512])
def test_flash_fwd_bwd(dt, D, causal, N):
    _check_flash(dt, D, causal, N, 2, 3)


@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("causal", [False, True])
@pytest.mark.parametrize("N", [128, 200, 512])
def test_flash_fwd_bwd_d80_native(dt, causal, N):
    """d_head 80 (the 2.7b model) runs natively (96-wide inside the kernel), no host padding."""
    from cs336_systems.ops.flash_attention import _padded_d

    assert _padded_d(80, dt) == 80
    _check_flash(dt, 80, causal, N, 2, 3)


@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("causal", [False, True])
@pytest.mark.parametrize("N", [128, 200, 512, 1100])
def test_flash_fwd_bwd_d16_native(dt, causal, N, monkeypatch):
    """d_head 16 (the reference's attention sweeps) runs natively (32-wide inside the kernel: no
    F.pad copies of q/k/v/dO and no slicing of O / the gradients on the host)."""
    from cs336_systems.ops.flash_attention import _padded_d

    assert _padded_d(16, dt) == 16
    _check_flash(dt, 16, causal, N, 2, 3)
    monkeypatch.setenv("CS336_FA_DMA", "2")  # the LDS-DMA staging with the 2 real chunks of 4
    _check_flash(dt, 16, causal, N, 1, 2)


@pytest.mark.parametrize("D", [64, 128])
@pytest.mark.parametrize("causal", [False, True])
@pytest.mark.parametrize("N", [200, 512])
@pytest.mark.parametrize("B,H", [(2, 4), (4, 6)])
def test_flash_fwd_bwd_xcd_head_ranges(D, causal, N, B, H):
    """B*H % 8 == 0: the causal grid takes the per-XCD head-range LPT order of tile_order
    (csrc/flash_attn/fa_common.h); B*H = 6 above takes the global level-major form."""
    _check_flash(torch.bfloat16, D, causal, N, B, H)


def _check_flash(dt, D, causal, N, B, H):
    torch.manual_seed(0)
    # (B, N, H, D) memory viewed as (B, H, N, D): the model's layout
    mk = lambda: torch.randn(B, N, H, D, device=DEV, dtype=dt).transpose(1, 2).requires_grad_(True)
    q, k, v = mk(), mk(), mk()
    o = ops.FlashAttentionHIP.apply(q, k, v, causal)
    assert o.dtype == dt
    o_ref, L_ref = _ref_attn(q.detach(), k.detach(), v.detach(), causal)
    tol = 2e-3 if dt == torch.float32 else 2e-2
    torch.testing.assert_close(o.double(), o_ref, rtol=tol, atol=tol)
    L = [t for t in o.grad_fn.saved_tensors if t.shape == (B, H, N)]
    assert len(L) == 1
    torch.testing.assert_close(L[0].double(), L_ref, rtol=1e-3, atol=1e-3)
    do = torch.randn_like(o)
    o.backward(do)
    qr, kr, vr = (t.detach().double().requires_grad_(True) for t in (q, k, v))
    orr, _ = _ref_attn(qr, kr, vr, causal)
    orr.backward(do.double())
    gt = 5e-3 if dt == torch.float32 else 5e-2
    for a, b in ((q.grad, qr.grad), (k.grad, kr.grad), (v.grad, vr.grad)):
        torch.testing.assert_close(a.double(), b, rtol=gt, atol=gt)


def test_flash_fwd_bwd_d16_padded():
    torch.manual_seed(0)
    q, k, v = (torch.randn(2, 96, 16, device=DEV, requires_grad=True) for _ in range(3))
    o = ops.FlashAttentionHIP.apply(q, k, v, True)
    o_ref, _ = _ref_attn(q.detach(), k.detach(), v.detach(), True)
    torch.testing.assert_close(o.double(), o_ref, rtol=2e-3, atol=2e-3)
    o.sum().backward()
    assert q.grad.shape == q.shape


def test_flash_rescale_branch_spike():
    """Force the online-softmax rescale: one key spikes against every query at a late tile."""
    torch.manual_seed(0)
    B, N, D = 1, 512, 64
    q = torch.randn(B, N, D, device=DEV, dtype=torch.bfloat16)
    k = torch.randn(B, N, D, device=DEV, dtype=torch.bfloat16)
    v = torch.randn(B, N, D, device=DEV, dtype=torch.bfloat16)
    k[:, 300] = 4 * q.mean(1)  # large score for many queries at tile 4
    o = ops.FlashAttentionHIP.apply(q, k, v, False)
    o_ref, _ = _ref_attn(q, k, v, False)
    torch.testing.assert_close(o.double(), o_ref, rtol=3e-2, atol=3e-2)


# ---------------------------------------------------------------------------------- model
def test_model_gpu_matches_cpu_reference():
    from cs336_systems.models import BasicsTransformerLM

    torch.manual_seed(0)
    m = BasicsTransformerLM(1000, 64, 128, 2, 4, 256, 10000.0)
    x = torch.randint(0, 1000, (2, 64))
    with ops.backend("torch"):
        ref = m(x)
    mg = m.to(DEV)
    out = mg(x.to(DEV))
    torch.testing.assert_close(out.cpu(), ref, rtol=2e-3, atol=2e-3)
    loss = ops.cross_entropy(out, x.to(DEV))
    loss.backward()
    assert all(p.grad is not None and torch.isfinite(p.grad).all() for p in mg.parameters())


def test_model_bf16_autocast_step():
    from cs336_systems.models import build_model

    torch.manual_seed(0)
    m = build_model("tiny", 128, device=DEV)
    opt = ops.FusedAdamW(m.parameters(), lr=1e-3)
    x = torch.randint(0, 10000, (4, 128), device=DEV)
    losses = []
    for _ in range(5):
        opt.zero_grad(set_to_none=True)
        with torch.autocast("cuda", dtype=torch.bfloat16):
            loss = ops.cross_entropy(m(x), x)
        loss.backward()
        opt.step()
        losses.append(loss.item())
    assert losses[-1] < losses[0]


# ---------------------------------------------------------------------------------- fused layout
def test_swiglu_fused_matches_reference():
    from cs336_systems.models.fused import SwiGLUGate

    torch.manual_seed(0)
    F = 384
    y = torch.randn(5, 7, 2 * F, device=DEV, dtype=torch.bfloat16, requires_grad=True)
    h = SwiGLUGate.apply(y)
    yr = y.detach().float().requires_grad_(True)
    hr = ops.silu_mul_ref(yr[..., :F], yr[..., F:])
    torch.testing.assert_close(h.float(), hr, rtol=2e-2, atol=2e-2)
    g = torch.randn_like(hr)
    h.backward(g.bfloat16())
    hr.backward(g.bfloat16().float())
    torch.testing.assert_close(y.grad.float(), yr.grad, rtol=3e-2, atol=3e-2)


@pytest.mark.parametrize("amp", [False, True])
@pytest.mark.parametrize("heads", [4, 2])
def test_fused_layout_matches_unfused(amp, heads):
    """Grouped QKV / W1|W3 GEMMs + AttentionCore + fp32-out dW == the unfused GPU path; heads=2 gives
    d_head 80 (the 2.7b model's): native 80-wide FA2 in the fused core under bf16 autocast, the
    host-padded FA2 through strided views in fp32."""
    from cs336_systems.models import BasicsTransformerLM

    torch.manual_seed(0)
    d = 256 if heads == 4 else 160
    cfg = dict(vocab_size=500, context_length=128, d_model=d, num_layers=2, num_heads=heads, d_ff=512, rope_theta=10000.0)
    m_f = BasicsTransformerLM(**cfg, device=DEV, fused_layout=True)
    m_u = BasicsTransformerLM(**cfg, device=DEV, fused_layout=False)
    m_u.load_state_dict(m_f.state_dict())
    from cs336_systems.models.fused import grouped_view

    assert grouped_view([m_f.layers[0].attn.q_proj.weight, m_f.layers[0].attn.k_proj.weight, m_f.layers[0].attn.v_proj.weight]) is not None
    assert grouped_view([m_u.layers[0].attn.q_proj.weight, m_u.layers[0].attn.k_proj.weight, m_u.layers[0].attn.v_proj.weight]) is None
    x = torch.randint(0, 500, (2, 128), device=DEV)
    outs = []
    for m in (m_f, m_u):
        with torch.autocast("cuda", dtype=torch.bfloat16, enabled=amp):
            loss = ops.cross_entropy(m(x), x)
        loss.backward()
        outs.append((loss.detach(), {n: p.grad for n, p in m.named_parameters()}))
    tol = 2e-2 if amp else 1e-3
    torch.testing.assert_close(outs[0][0], outs[1][0], rtol=tol, atol=tol)
    for n, g in outs[0][1].items():
        assert g.dtype == torch.float32
        torch.testing.assert_close(g, outs[1][1][n], rtol=5e-2 if amp else 2e-3, atol=5e-3 if amp else 1e-4, msg=n)


def test_bf16_shadows_track_master_weights():
    from cs336_systems.models import build_model
    from cs336_systems.models.fused import get_shadow, shadow_valid

    torch.manual_seed(0)
    m = build_model("tiny", 64, device=DEV)
    opt = ops.FusedAdamW(m.parameters(), lr=1e-2, bf16_shadows=True)
    w = m.layers[0].attn.q_proj.weight
    assert shadow_valid(w)
    assert torch.equal(get_shadow(w), w.detach().bfloat16())
    x = torch.randint(0, 10000, (2, 64), device=DEV)
    for _ in range(2):
        opt.zero_grad(set_to_none=True)
        with torch.autocast("cuda", dtype=torch.bfloat16):
            loss = ops.cross_entropy(m(x), x)
        loss.backward()
        opt.step()
        for p in m.parameters():
            if p.dim() == 2:
                assert shadow_valid(p)
                assert torch.equal(get_shadow(p), p.detach().bfloat16())
    with torch.no_grad():
        w.add_(1.0)  # out-of-band edit invalidates the shadow -> forward falls back to casting
    assert not shadow_valid(w)


# ---------------------------------------------------------------------------------- transpose
@pytest.mark.parametrize("shape", [(64, 64), (1600, 4800), (120, 72), (8, 200)])
@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float16])
def test_transpose2d(shape, dt):
    from cs336_systems.ops._ext import ops as _hip

    x = torch.randn(*shape, device=DEV).to(dt)
    torch.testing.assert_close(_hip().transpose2d(x), x.t().contiguous(), rtol=0, atol=0)
    big = torch.randn(shape[0], shape[1] + 16, device=DEV).to(dt)
    v = big[:, 8 : 8 + shape[1]]  # strided rows
    torch.testing.assert_close(_hip().transpose2d(v), v.t().contiguous(), rtol=0, atol=0)
