"""gemm8w (csrc/gemm/gemm8w.hip): weight gradients dW = dYᵀ·X straight from token-major bf16
operands, fp32 out (plain, transposed store, split-K slabs, accumulate), against an fp32 PyTorch
reference of the same product."""

import pytest
import torch

pytestmark = pytest.mark.gpu


def _cs():
    from cs336_systems import ops

    if not torch.cuda.is_available():
        pytest.skip("needs a GPU")
    assert ops.load_ext(), ops.load_error()
    return torch.ops.cs336


def _rand(*s, seed=0):
    g = torch.Generator(device="cuda").manual_seed(seed)
    return (torch.rand(*s, device="cuda", generator=g) * 2 - 1).to(torch.bfloat16)


def _rel(a, b):
    return float((a.float() - b.float()).norm() / b.float().norm().clamp_min(1e-30))


@pytest.mark.parametrize("K,M,N,trans,splits", [
    (64, 256, 320, False, 1), (192, 512, 640, False, 1), (128, 320, 640, False, 1),  # padded last row tile
    (256, 320, 320, True, 1), (512, 1600, 1600, False, 4), (384, 1600, 4800, True, 3), (128, 264, 256, False, 1),
    (1024, 512, 512, True, 2),
])
def test_gemm8w(K, M, N, trans, splits):
    cs = _cs()
    a, b = _rand(K, M, seed=1), _rand(K, N, seed=2)
    ref = a.float().t() @ b.float()
    shape = (N, M) if trans else (M, N)
    if splits > 1:
        out = torch.full((splits, *shape), float("nan"), device="cuda")
        cs.gemm8w(a, b, out, splits, trans, False, 0)
        got = out.sum(0)
    else:
        out = torch.full(shape, float("nan"), device="cuda")
        cs.gemm8w(a, b, out, 1, trans, False, 0)
        got = out
    if trans:
        got = got.t()
    assert torch.isfinite(got).all()
    assert _rel(got, ref) < 1e-5, _rel(got, ref)


def test_gemm8w_strided_accumulate_bucket_view():
    """Operands with row strides wider than their width (the fused QKV output), output written into
    a row block of a larger fp32 buffer (a DDP bucket) and accumulated."""
    cs = _cs()
    K, M, N = 256, 960, 640
    abuf, bbuf = _rand(K, M + 320, seed=3), _rand(K, N + 64, seed=4)
    a, b = abuf[:, 320:], bbuf[:, :N]
    bucket = torch.zeros(M * N + 4096, device="cuda")
    out = bucket[1024: 1024 + M * N].view(M, N)
    out.fill_(1.0)
    cs.gemm8w(a, b, out, 1, False, True, 0)
    ref = a.float().t() @ b.float() + 1.0
    assert _rel(out, ref) < 1e-5
    assert torch.count_nonzero(bucket[:1024]) == 0 and torch.count_nonzero(bucket[1024 + M * N:]) == 0


def test_gemm8w_xl_w13():
    """The XL W1|W3 weight gradient at the bench's 24576 tokens (K = tokens, M = 12800, N = 1600)."""
    cs = _cs()
    T = 24576
    dy, x = _rand(T, 12800, seed=5), _rand(T, 1600, seed=6)
    out = torch.empty(12800, 1600, device="cuda")
    cs.gemm8w(dy, x, out, 1, False, False, 0)
    ref = torch.mm(dy.t(), x, out_dtype=torch.float32)
    assert _rel(out, ref) < 1e-4


def test_gemm8w_past_2gib_chunked():
    """A dY whose extent passes the kernel's 2 GiB DMA range (row stride of a 50304-column buffer,
    49152 tokens = 4.9 GB): the binding cuts the token range into chunks that accumulate; split-K
    plans that would overflow fall back to one split."""
    from cs336_systems.ops import gemm

    cs = _cs()
    T, V, d = 49152, 50304, 256
    buf = torch.empty(T, V, device="cuda", dtype=torch.bfloat16)
    dy = buf[:, :512]
    dy.copy_(_rand(T, 512, seed=7))
    x = _rand(T, d, seed=8)
    out = torch.full((512, d), float("nan"), device="cuda")
    cs.gemm8w(dy, x, out, 1, False, False, 0)
    ref = torch.mm(dy.t(), x, out_dtype=torch.float32)
    assert _rel(out, ref) < 1e-4
    with pytest.raises(RuntimeError, match="2 GiB"):
        cs.gemm8w(dy, x, torch.empty(2, 512, d, device="cuda"), 2, False, False, 0)  # 24576 rows x 100 KB
    got = gemm.mm_dw(dy, x)  # plan + fallback through the Python path
    assert _rel(got, ref) < 1e-4
    del buf
