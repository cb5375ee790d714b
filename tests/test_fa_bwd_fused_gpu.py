"""The one-kernel FlashAttention-2 backwards (csrc/flash_attn/fa_bwd_fused.hip: one 8-wave workgroup
per (batch, head); fa_bwd_hs.hip: one 4-wave workgroup per (batch, head), two per CU; fa_bwd_kp.hip:
one workgroup per key block, dQ by per-key-block slabs or atomics) against an fp64 reference, the two-kernel backward, and
the default selection (head-sequential at B·H >= 512)."""

import math

import pytest
import torch

from cs336_systems.models import RotaryEmbedding
from cs336_systems.ops._ext import ops as _hip

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _ref(q, k, v, do, causal):
    qr, kr, vr = (t.detach().double().requires_grad_(True) for t in (q, k, v))
    s = qr @ kr.transpose(-1, -2) / math.sqrt(q.shape[-1])
    if causal:
        n = q.shape[-2]
        s = s.masked_fill(~torch.ones(n, n, dtype=torch.bool, device=q.device).tril(), float("-inf"))
    o = torch.softmax(s, -1) @ vr
    o.backward(do.double())
    return qr.grad, kr.grad, vr.grad


def _inputs(B, H, N, dt, seed=0):
    torch.manual_seed(seed)
    mk = lambda: torch.randn(B, N, H, 64, device=DEV, dtype=dt).transpose(1, 2)  # noqa: E731
    return mk(), mk(), mk(), mk()


@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("causal", [True, False])
@pytest.mark.parametrize("N", [64, 128, 256, 320, 512, 768, 1024])
def test_fused_bwd_vs_fp64(dt, causal, N, monkeypatch):
    monkeypatch.setenv("CS336_FA_BWD", "1")
    B, H = 2, 3
    q, k, v, do = _inputs(B, H, N, dt)
    hip = _hip()
    o, lse = hip.fa_fwd(q, k, v, causal, 0.125)
    dq, dk, dv = hip.fa_bwd(do, q, k, v, o, lse, causal, 0.125)
    rq, rk, rv = _ref(q, k, v, do, causal)
    for a, b, name in ((dq, rq, "dq"), (dk, rk, "dk"), (dv, rv, "dv")):
        err = (a.double() - b).abs().max().item()
        scale = b.abs().max().item()
        assert err <= 2e-2 * max(1.0, scale), f"{name}: max err {err} (ref max {scale})"


@pytest.mark.parametrize("causal", [True, False])
@pytest.mark.parametrize("N", [256, 512, 1024])
def test_fused_matches_two_kernel(causal, N, monkeypatch):
    B, H = 3, 5
    q, k, v, do = _inputs(B, H, N, torch.bfloat16, seed=1)
    hip = _hip()
    o, lse = hip.fa_fwd(q, k, v, causal, 0.125)
    monkeypatch.setenv("CS336_FA_BWD", "0")
    two = hip.fa_bwd(do, q, k, v, o, lse, causal, 0.125)
    monkeypatch.setenv("CS336_FA_BWD", "1")
    fused = hip.fa_bwd(do, q, k, v, o, lse, causal, 0.125)
    again = hip.fa_bwd(do, q, k, v, o, lse, causal, 0.125)
    for a, b, c in zip(fused, two, again):
        assert torch.equal(a, c)  # deterministic: no atomics
        torch.testing.assert_close(a.float(), b.float(), rtol=2e-2, atol=2e-2)


def test_fused_rope_out_only_in_step_layout(monkeypatch):
    """The XL step's call: dq/dk/dv written into the three slices of one fused d(qkv) buffer, q/k
    already rotated, dq/dk returned w.r.t. the un-rotated inputs; B·H = 600 >= 512 takes the
    head-sequential two-workgroups-per-CU kernel by default (bitwise equal to forcing it), and the
    8-wave fused kernel agrees with the two-kernel form."""
    B, H, N, D = 24, 25, 512, 64
    torch.manual_seed(2)
    qkv = torch.randn(B, N, 3, H, D, device=DEV, dtype=torch.bfloat16)
    q, k, v = qkv[:, :, 0].transpose(1, 2), qkv[:, :, 1].transpose(1, 2), qkv[:, :, 2].transpose(1, 2)
    do = torch.randn(B, N, H, D, device=DEV, dtype=torch.bfloat16).transpose(1, 2)
    re = RotaryEmbedding(1024, D, 10000.0).to(DEV)
    cos, sin = re.cos.contiguous(), re.sin.contiguous()
    hip = _hip()
    o, lse = hip.fa_fwd(q, k, v, True, D**-0.5)

    def run():
        d = torch.empty(B, N, 3, H, D, device=DEV, dtype=torch.bfloat16)
        dq, dk, dv = d[:, :, 0].transpose(1, 2), d[:, :, 1].transpose(1, 2), d[:, :, 2].transpose(1, 2)
        hip.fa_bwd_into(do, q, k, v, o, lse, True, D**-0.5, dq, dk, dv, cos, sin, None, True)
        return d

    monkeypatch.delenv("CS336_FA_BWD", raising=False)
    monkeypatch.delenv("CS336_FA_HS_ROPE", raising=False)
    default = run()
    monkeypatch.setenv("CS336_FA_BWD", "3")
    hs = run()
    monkeypatch.setenv("CS336_FA_BWD", "1")
    fused = run()
    monkeypatch.setenv("CS336_FA_BWD", "0")
    two = run()
    assert torch.equal(default, hs)
    torch.testing.assert_close(fused.float(), two.float(), rtol=2e-2, atol=2e-2)
    torch.testing.assert_close(hs.float(), two.float(), rtol=2e-2, atol=2e-2)


# ---- key-block-parallel fused backward (csrc/flash_attn/fa_bwd_kp.hip, dQ by per-key-block fp32
# slabs; fp32 atomics past 4 GiB of slabs or with CS336_FA_KP_SLAB=0) ----
def _inputs_d(B, H, N, D, dt, seed=0):
    torch.manual_seed(seed)
    mk = lambda: torch.randn(B, N, H, D, device=DEV, dtype=dt).transpose(1, 2)  # noqa: E731
    return mk(), mk(), mk(), mk()


@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("causal", [True, False])
@pytest.mark.parametrize("N,D", [(64, 64), (256, 64), (320, 64), (512, 64), (1024, 64), (2048, 64),
                                 (64, 80), (320, 80), (1024, 80)])
@pytest.mark.parametrize("waves", [4, 8])
def test_kp_bwd_vs_fp64(dt, causal, N, D, waves, monkeypatch):
    monkeypatch.setenv("CS336_FA_BWD", "2")
    monkeypatch.setenv("CS336_FA_KP_WAVES", str(waves))
    B, H = 2, 3
    q, k, v, do = _inputs_d(B, H, N, D, dt)
    hip = _hip()
    sc = D**-0.5
    o, lse = hip.fa_fwd(q, k, v, causal, sc)
    dq, dk, dv = hip.fa_bwd(do, q, k, v, o, lse, causal, sc)
    rq, rk, rv = _ref(q, k, v, do, causal)
    for a, b, name in ((dq, rq, "dq"), (dk, rk, "dk"), (dv, rv, "dv")):
        assert torch.isfinite(a).all(), name
        err = (a.double() - b).abs().max().item()
        scale = b.abs().max().item()
        assert err <= 2e-2 * max(1.0, scale), f"{name}: max err {err} (ref max {scale})"


@pytest.mark.parametrize("causal", [True, False])
@pytest.mark.parametrize("N,D", [(320, 80), (1024, 80), (2048, 64)])
def test_kp_slabs_vs_atomics(causal, N, D, monkeypatch):
    """dQ summed from per-key-block slabs (the default up to N 1024, forced here) equals the atomic
    accumulation up to fp32 add order, is bitwise reproducible run to run, and leaves dK / dV bitwise
    unchanged."""
    monkeypatch.setenv("CS336_FA_BWD", "2")
    monkeypatch.setenv("CS336_FA_KP_SLAB", "1")
    B, H = 2, 3
    q, k, v, do = _inputs_d(B, H, N, D, torch.bfloat16, seed=5)
    hip = _hip()
    sc = D**-0.5
    o, lse = hip.fa_fwd(q, k, v, causal, sc)
    slab = hip.fa_bwd(do, q, k, v, o, lse, causal, sc)
    again = hip.fa_bwd(do, q, k, v, o, lse, causal, sc)
    monkeypatch.setenv("CS336_FA_KP_SLAB", "0")
    atom = hip.fa_bwd(do, q, k, v, o, lse, causal, sc)
    for a, b in zip(slab, again):
        assert torch.equal(a, b)
    assert torch.equal(slab[1], atom[1]) and torch.equal(slab[2], atom[2])
    torch.testing.assert_close(slab[0].float(), atom[0].float(), rtol=1e-2, atol=1e-2)
    rq, _, _ = _ref(q, k, v, do, causal)
    for a in (slab[0], atom[0]):
        err = (a.double() - rq).abs().max().item()
        assert err <= 2e-2 * max(1.0, rq.abs().max().item())


@pytest.mark.parametrize("causal", [True, False])
@pytest.mark.parametrize("D", [64, 80])
@pytest.mark.parametrize("waves", [4, 8])
def test_kp_matches_two_kernel_long(causal, D, waves, monkeypatch):
    """The reference FA benchmark's regime: few heads, long N (B·H 8, N 4096)."""
    B, H, N = 2, 4, 4096
    q, k, v, do = _inputs_d(B, H, N, D, torch.bfloat16, seed=3)
    hip = _hip()
    o, lse = hip.fa_fwd(q, k, v, causal, D**-0.5)
    monkeypatch.setenv("CS336_FA_BWD", "0")
    two = hip.fa_bwd(do, q, k, v, o, lse, causal, D**-0.5)
    monkeypatch.setenv("CS336_FA_BWD", "2")  # key-block parallel (the default only at d 80)
    monkeypatch.setenv("CS336_FA_KP_WAVES", str(waves))
    kp = hip.fa_bwd(do, q, k, v, o, lse, causal, D**-0.5)
    for a, b in zip(kp, two):
        torch.testing.assert_close(a.float(), b.float(), rtol=2e-2, atol=2e-2)


@pytest.mark.parametrize("causal", [True, False])
def test_default_long_d64_selects_kp(causal, monkeypatch):
    """At d 64, N >= 2048 with >= 512 key-block workgroups the default backward is the 8-wave
    key-block-parallel kernel (csrc/bindings.cpp): it must match the two-kernel form there."""
    B, H, N, D = 4, 16, 4096, 64
    q, k, v, do = _inputs_d(B, H, N, D, torch.bfloat16, seed=6)
    hip = _hip()
    o, lse = hip.fa_fwd(q, k, v, causal, D**-0.5)
    monkeypatch.delenv("CS336_FA_BWD", raising=False)
    default = hip.fa_bwd(do, q, k, v, o, lse, causal, D**-0.5)
    monkeypatch.setenv("CS336_FA_BWD", "2")
    kp = hip.fa_bwd(do, q, k, v, o, lse, causal, D**-0.5)
    monkeypatch.setenv("CS336_FA_BWD", "0")
    two = hip.fa_bwd(do, q, k, v, o, lse, causal, D**-0.5)
    for a, b, c in zip(default, kp, two):
        # dK / dV have no atomics: the default is the key-block-parallel kernel bit for bit
        torch.testing.assert_close(a.float(), c.float(), rtol=2e-2, atol=2e-2)
    assert torch.equal(default[1], kp[1]) and torch.equal(default[2], kp[2])


@pytest.mark.parametrize("D", [64, 80])
def test_kp_rope_out_only_in_step_layout(D, monkeypatch):
    """The 2.7b step's call shape: strided views of one fused d(qkv) buffer, q/k already rotated,
    dq/dk returned w.r.t. the un-rotated inputs (dK rotated back in its store, dQ in the convert)."""
    B, H, N = 3, 4, 1024
    torch.manual_seed(4)
    qkv = torch.randn(B, N, 3, H, D, device=DEV, dtype=torch.bfloat16)
    q, k, v = qkv[:, :, 0].transpose(1, 2), qkv[:, :, 1].transpose(1, 2), qkv[:, :, 2].transpose(1, 2)
    do = torch.randn(B, N, H, D, device=DEV, dtype=torch.bfloat16).transpose(1, 2)
    re = RotaryEmbedding(2048, D, 10000.0).to(DEV)
    cos, sin = re.cos.contiguous(), re.sin.contiguous()
    hip = _hip()
    o, lse = hip.fa_fwd(q, k, v, True, D**-0.5)

    def run():
        d = torch.empty(B, N, 3, H, D, device=DEV, dtype=torch.bfloat16)
        dq, dk, dv = d[:, :, 0].transpose(1, 2), d[:, :, 1].transpose(1, 2), d[:, :, 2].transpose(1, 2)
        hip.fa_bwd_into(do, q, k, v, o, lse, True, D**-0.5, dq, dk, dv, cos, sin, None, True)
        return d

    monkeypatch.setenv("CS336_FA_BWD", "2")
    kp = run()
    monkeypatch.setenv("CS336_FA_BWD", "0")
    two = run()
    torch.testing.assert_close(kp.float(), two.float(), rtol=2e-2, atol=2e-2)


# ---- head-sequential backward, two 4-wave workgroups per CU (csrc/flash_attn/fa_bwd_hs.hip) ----
@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("causal", [True, False])
@pytest.mark.parametrize("N", [128, 256, 384, 512, 1024, 2048])
def test_hs_bwd_vs_fp64(dt, causal, N, monkeypatch):
    monkeypatch.setenv("CS336_FA_BWD", "3")
    B, H = 2, 3
    q, k, v, do = _inputs(B, H, N, dt)
    hip = _hip()
    o, lse = hip.fa_fwd(q, k, v, causal, 0.125)
    dq, dk, dv = hip.fa_bwd(do, q, k, v, o, lse, causal, 0.125)
    again = hip.fa_bwd(do, q, k, v, o, lse, causal, 0.125)
    rq, rk, rv = _ref(q, k, v, do, causal)
    for a, b, c, name in ((dq, rq, again[0], "dq"), (dk, rk, again[1], "dk"), (dv, rv, again[2], "dv")):
        assert torch.equal(a, c), name  # deterministic: no atomics
        err = (a.double() - b).abs().max().item()
        scale = b.abs().max().item()
        assert err <= 2e-2 * max(1.0, scale), f"{name}: max err {err} (ref max {scale})"


@pytest.mark.parametrize("rope_in_kernel", ["1", "0", "2"])
def test_hs_rope_out_only_in_step_layout(rope_in_kernel, monkeypatch):
    """The XL step's call through the two-workgroups-per-CU kernel: strided views of one fused
    d(qkv) buffer, q/k already rotated, the inverse RoPE in the dQ / dK stores (or the separate pass)."""
    B, H, N, D = 6, 25, 512, 64
    torch.manual_seed(5)
    qkv = torch.randn(B, N, 3, H, D, device=DEV, dtype=torch.bfloat16)
    q, k, v = qkv[:, :, 0].transpose(1, 2), qkv[:, :, 1].transpose(1, 2), qkv[:, :, 2].transpose(1, 2)
    do = torch.randn(B, N, H, D, device=DEV, dtype=torch.bfloat16).transpose(1, 2)
    re = RotaryEmbedding(1024, D, 10000.0).to(DEV)
    cos, sin = re.cos.contiguous(), re.sin.contiguous()
    hip = _hip()
    o, lse = hip.fa_fwd(q, k, v, True, D**-0.5)

    def run():
        d = torch.empty(B, N, 3, H, D, device=DEV, dtype=torch.bfloat16)
        dq, dk, dv = d[:, :, 0].transpose(1, 2), d[:, :, 1].transpose(1, 2), d[:, :, 2].transpose(1, 2)
        hip.fa_bwd_into(do, q, k, v, o, lse, True, D**-0.5, dq, dk, dv, cos, sin, None, True)
        return d

    monkeypatch.setenv("CS336_FA_HS_ROPE", rope_in_kernel)
    monkeypatch.setenv("CS336_FA_BWD", "3")
    hs = run()
    monkeypatch.setenv("CS336_FA_BWD", "0")
    two = run()
    torch.testing.assert_close(hs.float(), two.float(), rtol=2e-2, atol=2e-2)


@pytest.mark.parametrize("causal", [True, False])
@pytest.mark.parametrize("N", [128, 512, 1024])
def test_hs_in_kernel_delta_matches_prep(causal, N, monkeypatch):
    """fa_bwd_hs.hip computes delta = rowsum(dO·O) itself during the first key block (default for
    N <= 1024) or takes it from the prep kernel (CS336_FA_HS_DELTA=0): same sums, bitwise equal."""
    monkeypatch.setenv("CS336_FA_BWD", "3")
    B, H = 3, 4
    q, k, v, do = _inputs(B, H, N, torch.bfloat16, seed=6)
    hip = _hip()
    o, lse = hip.fa_fwd(q, k, v, causal, 0.125)
    ind = hip.fa_bwd(do, q, k, v, o, lse, causal, 0.125)
    monkeypatch.setenv("CS336_FA_HS_DELTA", "0")
    prep = hip.fa_bwd(do, q, k, v, o, lse, causal, 0.125)
    for a, b in zip(ind, prep):
        assert torch.equal(a, b)
