"""FA2 forward that also writes Oᵀ (csrc/flash_attn/fa_fwd.hip, `fa_fwd_ot`), consumed as the
token-contiguous operand of the output projection's weight gradient (models/fused.py)."""

import pytest
import torch

from cs336_systems import ops

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.mark.parametrize("D", [64, 80, 128])
@pytest.mark.parametrize("N", [200, 512])
def test_fa_fwd_ot_is_transposed_o(D, N, monkeypatch):
    assert ops.load_ext(), ops.load_error()
    torch.manual_seed(0)
    B, H = 2, 3
    mk = lambda: torch.randn(B, N, H, D, device=DEV, dtype=torch.bfloat16).transpose(1, 2)  # noqa: E731
    q, k, v = mk(), mk(), mk()
    # fa_fwd_ot never splits over the keys; at this low parallelism fa_fwd would (N 512: 8 key tiles),
    # which rounds differently: compare bitwise with the split off, and closely with it on
    o_split, lse_split = torch.ops.cs336.fa_fwd(q, k, v, True, D**-0.5)
    monkeypatch.setenv("CS336_FA_SPLITS", "1")
    o, lse = torch.ops.cs336.fa_fwd(q, k, v, True, D**-0.5)
    o2, lse2, ot = torch.ops.cs336.fa_fwd_ot(q, k, v, True, D**-0.5)
    assert torch.equal(o, o2) and torch.equal(lse, lse2)
    torch.testing.assert_close(o_split.float(), o.float(), atol=2e-2, rtol=2e-2)
    torch.testing.assert_close(lse_split, lse, atol=1e-4, rtol=1e-5)
    # (B, H, N, D) -> (H*D, B*N)
    ref = o.permute(1, 3, 0, 2).reshape(H * D, B * N)
    assert ot.shape == (H * D, B * N) and torch.equal(ot, ref)


def test_model_grads_with_and_without_ot(monkeypatch):
    from cs336_systems.models import BasicsTransformerLM

    grads = []
    for flag in ("1", "0"):
        monkeypatch.setenv("CS336_OT", flag)
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


@pytest.mark.parametrize("D", [64, 80, 128])
def test_fa_bwd_rope_out_only_matches_separate_inverse(D):
    """fa_bwd_into(..., rope_out_only=True) on already-rotated q/k returns dq/dk w.r.t. the
    un-rotated inputs: same as the plain backward followed by rope_into(inverse)."""
    assert ops.load_ext(), ops.load_error()
    torch.manual_seed(0)
    B, H, N = 2, 3, 320
    mk = lambda: torch.randn(B, N, H, D, device=DEV, dtype=torch.bfloat16).transpose(1, 2)  # noqa: E731
    q, k, v, do = mk(), mk(), mk(), mk()
    pos = torch.arange(N, device=DEV).flip(0).repeat(B, 1).contiguous()  # non-trivial positions
    theta = 10000.0 ** (-torch.arange(0, D, 2, device=DEV).float() / D)
    ang = torch.arange(1024, device=DEV).float()[:, None] * theta[None]
    cos, sin = ang.cos().contiguous(), ang.sin().contiguous()
    scale = D**-0.5
    o, lse = torch.ops.cs336.fa_fwd(q, k, v, True, scale)
    outs = []
    for fused_mode in (True, False):
        dq, dk, dv = (torch.empty(B, N, H, D, device=DEV, dtype=torch.bfloat16).transpose(1, 2) for _ in range(3))
        if fused_mode:
            torch.ops.cs336.fa_bwd_into(do, q, k, v, o, lse, True, scale, dq, dk, dv, cos, sin, pos, True)
        else:
            torch.ops.cs336.fa_bwd_into(do, q, k, v, o, lse, True, scale, dq, dk, dv)
            torch.ops.cs336.rope_into(dq, cos, sin, pos, True, dq)
            torch.ops.cs336.rope_into(dk, cos, sin, pos, True, dk)
        outs.append((dq.float(), dk.float(), dv.float()))
    for a, b, name in zip(outs[0], outs[1], ("dq", "dk", "dv")):
        err = float((a - b).norm() / b.norm())
        assert err < 1e-2, f"{name}: {err:.2e}"


def test_model_grads_rope_out_in_fa(monkeypatch):
    from cs336_systems.models import BasicsTransformerLM

    grads = []
    for flag in ("1", "0"):
        monkeypatch.setenv("CS336_FA_ROPE_OUT", flag)
        torch.manual_seed(0)
        m = BasicsTransformerLM(vocab_size=512, context_length=128, d_model=256, num_layers=2, num_heads=4, d_ff=512,
                                device=DEV)
        x = torch.randint(0, 512, (4, 128), device=DEV, generator=torch.Generator(DEV).manual_seed(1))
        with torch.autocast("cuda", dtype=torch.bfloat16):
            loss = ops.cross_entropy(m(x), x)
        loss.backward()
        grads.append({n: p.grad.clone() for n, p in m.named_parameters()})
    worst = {}
    for n, g in grads[0].items():
        worst[n] = float((g - grads[1][n]).norm() / grads[1][n].norm().clamp_min(1e-30))
    # one bf16 rounding of dQ/dK (fused) vs two (separate pass): ~1e-3 relative on the grads
    assert max(worst.values()) < 1e-2, sorted(worst.items(), key=lambda kv: -kv[1])[:4]
