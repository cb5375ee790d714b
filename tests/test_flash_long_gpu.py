"""FlashAttention-2 numerics at the benchmarked shapes.

The short-sequence tests (test_kernels_gpu.py, N <= 512) never reach the long-N code paths the
benchmarks time: many query blocks under the causal LPT block order, the per-XCD head ranges
(B*H % 8 == 0), the L2-sized head groups of that order, and the deferred online-softmax rescale
over dozens of key tiles. Here forward (O, LSE) and backward (dQ, dK, dV) are checked against an
fp32 PyTorch reference computed one head and one block of queries at a time:

* BASELINE config 2: N = 4096, d_head 64 and 128, causal and not, bf16, B*H = 8;
* the handout leaderboard shape (16, 16384, 64) causal bf16, compared on a subset of its heads.

Errors are relative Frobenius norms (bf16 inputs and outputs: ~4e-3 is typical).
"""

import math

import pytest
import torch

pytestmark = pytest.mark.gpu

DEV = "cuda"


def _ops():
    from cs336_systems import ops

    if not torch.cuda.is_available():
        pytest.skip("needs a GPU")
    assert ops.load_ext(), ops.load_error()
    return ops


def _ref_head(q, k, v, do, causal, chunk=1024):
    """fp32 reference for one head: q,k,v,do (N, D) -> o, lse, dq, dk, dv (blocks of queries)."""
    q, k, v, do = (t.float() for t in (q, k, v, do))
    N, D = q.shape
    scale = 1.0 / math.sqrt(D)
    o = torch.empty_like(q)
    lse = torch.empty(N, device=q.device)
    dq = torch.empty_like(q)
    dk = torch.zeros_like(k)
    dv = torch.zeros_like(v)
    keys = torch.arange(N, device=q.device)
    for s in range(0, N, chunk):
        e = min(N, s + chunk)
        sc = (q[s:e] @ k.t()) * scale
        if causal:
            sc = sc.masked_fill(keys[None, :] > torch.arange(s, e, device=q.device)[:, None], float("-inf"))
        L = torch.logsumexp(sc, -1)
        p = torch.exp(sc - L[:, None])
        o[s:e] = p @ v
        lse[s:e] = L
        delta = (do[s:e] * o[s:e]).sum(-1, keepdim=True)
        dp = do[s:e] @ v.t()
        ds = p * (dp - delta)
        dq[s:e] = ds @ k * scale
        dk += ds.t() @ q[s:e] * scale
        dv += p.t() @ do[s:e]
    return o, lse, dq, dk, dv


def _rel(a, b):
    return float((a.float() - b.float()).norm() / b.float().norm().clamp_min(1e-30))


def _run(B, H, N, D, causal, heads_to_check):
    ops = _ops()
    torch.manual_seed(0)
    # (B, N, H, D) memory viewed as (B, H, N, D): the model's layout
    mk = lambda: torch.randn(B, N, H, D, device=DEV, dtype=torch.bfloat16).transpose(1, 2).requires_grad_(True)  # noqa: E731
    q, k, v = mk(), mk(), mk()
    o = ops.FlashAttentionHIP.apply(q, k, v, causal)
    (lse,) = [t for t in o.grad_fn.saved_tensors if t.shape == (B, H, N)]
    do = torch.randn_like(o)
    o.backward(do)
    worst = {}
    for (b, h) in heads_to_check:
        r = _ref_head(q[b, h].detach(), k[b, h].detach(), v[b, h].detach(), do[b, h], causal)
        got = (o[b, h], lse[b, h], q.grad[b, h], k.grad[b, h], v.grad[b, h])
        for name, g, ref in zip(("o", "lse", "dq", "dk", "dv"), got, r):
            worst[name] = max(worst.get(name, 0.0), _rel(g.detach(), ref))
    limits = dict(o=1e-2, lse=1e-4, dq=2e-2, dk=2e-2, dv=1e-2)
    for name, err in worst.items():
        assert err < limits[name], f"{name}: relative error {err:.2e} (limit {limits[name]:.0e}); all {worst}"


@pytest.mark.parametrize("causal", [True, False])
@pytest.mark.parametrize("D", [64, 128])
def test_flash_seq4096(D, causal):
    # B*H = 8: causal blocks take the per-XCD head-range LPT order; check one head per XCD range
    # at both ends of the grid
    _run(2, 4, 4096, D, causal, [(0, 0), (0, 3), (1, 1), (1, 3)])


def test_flash_leaderboard_shape_subset():
    """(16, 16384, 64) causal bf16 as (B=16, H=1): one head per XCD range end is checked."""
    _run(16, 1, 16384, 64, True, [(0, 0), (7, 0), (15, 0)])


@pytest.mark.parametrize("causal", [True, False])
@pytest.mark.parametrize("D", [64, 128])
def test_flash_seq4096_pipelined_forward(monkeypatch, D, causal):
    """CS336_FA_DMA=4: the software-pipelined forward (separate K/V LDS-DMA rings, next tile's S^T
    inside this tile's softmax) at the benchmarked shapes, plus a ragged length (partial last tile)."""
    monkeypatch.setenv("CS336_FA_DMA", "4")
    _run(2, 4, 4096, D, causal, [(0, 0), (1, 3)])
    _run(1, 2, 1000, D, causal, [(0, 0), (0, 1)])


@pytest.mark.parametrize("causal", [True, False])
@pytest.mark.parametrize("D", [64, 80, 128])
@pytest.mark.parametrize("N", [1100, 1500])
def test_flash_ragged_long_dma(D, N, causal):
    """LDS-DMA staging is the default for the backward at Nk >= 1024 and for the causal
    forward; a ragged Nk (Nk % BN != 0: zero-filled partial last tile) at those lengths, with the
    native d 80 path included, against the chunked fp32 reference."""
    _run(1, 2, N, D, causal, [(0, 0), (0, 1)])


@pytest.mark.parametrize("causal", [True, False])
@pytest.mark.parametrize("D", [64, 128])
def test_flash_dma_forced_short_ragged(monkeypatch, D, causal):
    """CS336_FA_DMA=2 (LDS-DMA forward AND backward) on short, ragged inputs, below the lengths where
    the default would choose it."""
    monkeypatch.setenv("CS336_FA_DMA", "2")
    _run(1, 2, 200, D, causal, [(0, 0), (0, 1)])
    _run(2, 1, 77, D, causal, [(0, 0), (1, 0)])


# ---- split-KV forward (low parallelism: the reference sweep's B 1, H 1) ----
@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float32])
@pytest.mark.parametrize("causal", [True, False])
@pytest.mark.parametrize("N,D", [(2048, 64), (4096, 128), (8192, 32), (1024, 16)])
def test_split_kv_forward_matches(dt, causal, N, D, monkeypatch):
    """B 1, H 1 takes the split-KV forward by default (partial O + LSE per key split, merged); it
    must match the unsplit kernel (CS336_FA_SPLITS=1) and an fp64 reference."""
    from cs336_systems.ops._ext import ops as hip_ops

    if dt == torch.float32 and D == 16:
        pytest.skip("d 16 is 16-bit only")
    torch.manual_seed(5)
    q, k, v = (torch.randn(1, 1, N, D, device="cuda", dtype=dt) for _ in range(3))
    hip = hip_ops()
    sc = D**-0.5
    monkeypatch.setenv("CS336_FA_SPLITS", "1")
    o1, l1 = hip.fa_fwd(q, k, v, causal, sc)
    monkeypatch.delenv("CS336_FA_SPLITS")
    o2, l2 = hip.fa_fwd(q, k, v, causal, sc)
    monkeypatch.setenv("CS336_FA_SPLITS", "7")  # uneven tile ranges, empty splits under the mask
    o3, l3 = hip.fa_fwd(q, k, v, causal, sc)
    s = (q.double() @ k.double().transpose(-1, -2)) * sc
    if causal:
        s = s.masked_fill(~torch.ones(N, N, dtype=torch.bool, device="cuda").tril(), float("-inf"))
    ref_l = torch.logsumexp(s, -1)
    ref_o = torch.softmax(s, -1) @ v.double()
    tol = 2e-2 if dt != torch.float32 else 1e-4
    for o, lse in ((o1, l1), (o2, l2), (o3, l3)):
        assert torch.isfinite(o).all()
        assert (o.double() - ref_o).abs().max().item() < tol
        assert (lse.double() - ref_l).abs().max().item() < tol
    torch.testing.assert_close(o2.float(), o1.float(), rtol=tol, atol=tol)


@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float32])
@pytest.mark.parametrize("causal", [True, False])
@pytest.mark.parametrize(
    "N,D", [(2048, 64), (4096, 128), (4096, 32), (1024, 16), (2048, 80), (256, 32), (512, 16), (384, 64), (1000, 64)]
)
def test_split_backward_matches(dt, causal, N, D, monkeypatch):
    """B 1, H 1: the two-kernel backward splits the dQ kernel over keys and the dK/dV kernel over
    queries into fp32 partial slabs, which ONE reduce launch (fa_bwd_reduce_kernel over SplitSum
    descriptors) sums for dQ, dK and dV; it must match the unsplit two-kernel form and fp64."""
    from cs336_systems.ops._ext import ops as hip_ops

    if dt == torch.float32 and D in (16, 80):
        pytest.skip("d 16 / 80 are 16-bit only")
    torch.manual_seed(6)
    q, k, v, do = (torch.randn(1, 1, N, D, device="cuda", dtype=dt) for _ in range(4))
    hip = hip_ops()
    sc = D**-0.5
    o, lse = hip.fa_fwd(q, k, v, causal, sc)
    monkeypatch.setenv("CS336_FA_BWD", "0")  # the two-kernel form (the split applies to it)
    monkeypatch.setenv("CS336_FA_BWD_SPLITS", "1")
    g1 = hip.fa_bwd(do, q, k, v, o, lse, causal, sc)
    monkeypatch.delenv("CS336_FA_BWD_SPLITS")
    g2 = hip.fa_bwd(do, q, k, v, o, lse, causal, sc)
    qr, kr, vr = (t.detach().double().requires_grad_(True) for t in (q, k, v))
    s = (qr @ kr.transpose(-1, -2)) * sc
    if causal:
        s = s.masked_fill(~torch.ones(N, N, dtype=torch.bool, device="cuda").tril(), float("-inf"))
    (torch.softmax(s, -1) @ vr).backward(do.double())
    tol = 2e-2 if dt != torch.float32 else 1e-3
    for a, b, r, name in zip(g2, g1, (qr.grad, kr.grad, vr.grad), ("dq", "dk", "dv")):
        assert torch.isfinite(a).all(), name
        err = (a.double() - r).abs().max().item()
        assert err <= tol * max(1.0, r.abs().max().item()), (name, err)
        torch.testing.assert_close(a.float(), b.float(), rtol=tol, atol=tol)
