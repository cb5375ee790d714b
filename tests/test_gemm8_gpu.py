"""gemm8 (csrc/gemm/gemm8.hip): the NT projection GEMM with fused SwiGLU epilogues, against an fp32
PyTorch reference of the same op (bf16 inputs, fp32 math, bf16-rounded where the kernel rounds)."""

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


def _rel(a, b):
    return float((a.float() - b.float()).norm() / b.float().norm().clamp_min(1e-30))


@pytest.mark.parametrize("M,N,K,fn", [(256, 320, 64, 0), (512, 640, 192, 5), (256, 512, 128, 4), (768, 1600, 1600, 0),
                                      (512, 1280, 320, 4), (256, 256, 4096, 0)])
def test_gemm8_plain(M, N, K, fn):
    cs = _cs()
    a, b = _rand(M, K, seed=1), _rand(N, K, seed=2)
    c = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
    cs.gemm8(a, b, c, 0, fn, None, None, 0)
    ref = a.float() @ b.float().t()
    assert _rel(c, ref) < 5e-3
    # exact tile placement: bf16 rounding of the fp32 sum, element by element
    torch.testing.assert_close(c.float(), ref.to(torch.bfloat16).float(), rtol=2e-2, atol=2e-2 * ref.abs().max().item() / 50)


def test_gemm8_strided_operands():
    """Row strides wider than K (views into wider buffers), as the fused QKV / Wᵀ layouts produce."""
    cs = _cs()
    M, N, K = 512, 640, 128
    abuf, bbuf = _rand(M, K + 64, seed=3), _rand(N, K + 192, seed=4)
    a, b = abuf[:, 32:32 + K], bbuf[:, :K]
    cbuf = torch.zeros(M, N + 64, device="cuda", dtype=torch.bfloat16)
    c = cbuf[:, 64:]
    cs.gemm8(a, b, c, 0, 0, None, None, 0)
    assert _rel(c, a.float() @ b.float().t()) < 5e-3
    assert torch.count_nonzero(cbuf[:, :64]) == 0


@pytest.mark.parametrize("half,fn", [(320, 5), (640, 0), (256, 4), (6400, 5)])
def test_gemm8_swiglu_forward(half, fn):
    cs = _cs()
    M, K = 512, 1600 if half == 6400 else 192
    x, w13 = _rand(M, K, seed=5), _rand(2 * half, K, scale=0.1, seed=6)
    y = torch.empty(M, 2 * half, device="cuda", dtype=torch.bfloat16)
    h = torch.empty(M, half, device="cuda", dtype=torch.bfloat16)
    cs.gemm8(x, w13, y, 1, fn, h, None, half)
    yr = x.float() @ w13.float().t()
    assert _rel(y, yr) < 5e-3
    yb = y.float()  # h is computed from the stored (bf16) a and b
    hr = torch.nn.functional.silu(yb[:, :half]) * yb[:, half:]
    assert _rel(h, hr) < 5e-3


@pytest.mark.parametrize("half,fn", [(320, 5), (640, 0), (256, 4), (6400, 5)])
def test_gemm8_swiglu_backward(half, fn):
    cs = _cs()
    M, K = 512, 1600 if half == 6400 else 192
    dy, w2t = _rand(M, K, seed=7), _rand(half, K, scale=0.1, seed=8)  # w2t = W2ᵀ (half, d_model)
    y = _rand(M, 2 * half, scale=3.0, seed=9)
    dab = torch.empty(M, 2 * half, device="cuda", dtype=torch.bfloat16)
    cs.gemm8(dy, w2t, dab, 2, fn, None, y, half)
    dh = dy.float() @ w2t.float().t()
    a, b = y.float()[:, :half], y.float()[:, half:]
    s = torch.sigmoid(a)
    da = dh * b * s * (1 + a * (1 - s))
    db = dh * a * s
    assert _rel(dab[:, :half], da) < 5e-3
    assert _rel(dab[:, half:], db) < 5e-3


def test_gemm8_xl_shapes():
    """The production shapes of the XL step (24576 tokens): QKV and W2 forward, W1|W3 input grad."""
    cs = _cs()
    M = 24576
    for N, K in ((4800, 1600), (1600, 6400), (1600, 12800)):
        a, b = _rand(M, K, seed=N), _rand(N, K, scale=0.05, seed=K)
        c = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
        cs.gemm8(a, b, c, 0, 0, None, None, 0)
        ref = torch.mm(a, b.t())  # hipBLASLt bf16 (fp32 accumulate)
        assert _rel(c, ref) < 5e-3, (N, K)


@pytest.mark.parametrize("M,N,K", [(256, 10000, 1600), (512, 1600, 10000), (256, 328, 72), (256, 88, 200),
                                   (768, 10000, 10000)])
def test_gemm8_tails(M, N, K):
    """N and K tails (multiples of 8; the vocabulary head's forward N = 10000 and input gradient
    K = 10000): out-of-range B rows and K chunks load as zeros, partial-tile stores are masked."""
    cs = _cs()
    a, b = _rand(M, K, seed=11), _rand(N, K, scale=0.1, seed=12)
    # NaN guards just past both operands (a K-tail chunk or B row read as data would poison C)
    abuf = torch.full((M + 1, K), float("nan"), device="cuda", dtype=torch.bfloat16)
    bbuf = torch.full((N + 1, K), float("nan"), device="cuda", dtype=torch.bfloat16)
    abuf[:M].copy_(a)
    bbuf[:N].copy_(b)
    cbuf = torch.zeros(M, N + 8, device="cuda", dtype=torch.bfloat16)
    c = cbuf[:, :N]
    cs.gemm8(abuf[:M], bbuf[:N], c, 0, 0, None, None, 0)
    ref = a.float() @ b.float().t()
    assert torch.isfinite(c.float()).all()
    assert _rel(c, ref) < 5e-3
    assert torch.count_nonzero(cbuf[:, N:]) == 0  # nothing stored past N


def test_gemm8_tail_strided():
    """K tail with a row stride wider than K (a padded buffer): the tail chunks read zeros, not the
    padding."""
    cs = _cs()
    M, N, K = 256, 1600, 10000
    abuf = torch.full((M, K + 48), 7.0, device="cuda", dtype=torch.bfloat16)
    a = abuf[:, :K]
    a.copy_(_rand(M, K, seed=13))
    b = _rand(N, K, scale=0.1, seed=14)
    c = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
    cs.gemm8(a, b, c, 0, 0, None, None, 0)
    assert _rel(c, a.float() @ b.float().t()) < 5e-3


@pytest.mark.parametrize("S,M,N,acc", [(4, 256, 320, False), (2, 1600, 1600, True), (8, 64, 2560, False)])
def test_splitk_sum(S, M, N, acc):
    """splitk_sum (the weight gradients' split-K slab reduction) against torch.sum in fp32, into a
    strided row-padded output, plain and accumulating."""
    cs = _cs()
    g = torch.Generator(device="cuda").manual_seed(1)
    slabs = torch.randn(S, M, N, device="cuda", generator=g)
    base = torch.randn(M, N + 4, device="cuda", generator=g)
    out = base.clone()
    view = out[:, :N]
    cs.splitk_sum(slabs, view, acc)
    ref = slabs.sum(0) + (base[:, :N] if acc else 0)
    torch.testing.assert_close(view, ref, rtol=1e-6, atol=1e-5)
    assert torch.equal(out[:, N:], base[:, N:])  # the row padding is untouched
