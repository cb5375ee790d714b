"""Autotuned hipBLASLt GEMM (``cs336::lt_gemm``, csrc/blas/lt_gemm.cpp) against an fp32 PyTorch
reference in every transpose combination and both output dtypes, strided (non-contiguous row
stride) operands and outputs, the tuned-problem table, and a model step under CS336_GEMM=lt."""

import pytest
import torch

from cs336_systems.ops._ext import ops

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _ref(a, b, a_t, b_t):
    A = a.float().t() if a_t else a.float()
    B = b.float().t() if b_t else b.float()
    return A @ B


@pytest.mark.parametrize("a_t,b_t", [(False, False), (False, True), (True, False), (True, True)])
@pytest.mark.parametrize("out_dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("M,N,K", [(256, 384, 512), (200, 136, 72), (1600, 480, 1024)])
def test_lt_gemm_matches_fp32(a_t, b_t, out_dtype, M, N, K):
    torch.manual_seed(0)
    a = torch.randn((K, M) if a_t else (M, K), device=DEV).bfloat16()
    b = torch.randn((N, K) if b_t else (K, N), device=DEV).bfloat16()
    out = ops().lt_gemm(a, b, a_t, b_t, out_dtype)
    assert out.dtype == out_dtype and out.shape == (M, N)
    ref = _ref(a, b, a_t, b_t)
    tol = 1e-3 if out_dtype == torch.float32 else 1e-2
    torch.testing.assert_close(out.float(), ref, rtol=tol, atol=tol * ref.abs().max().item())


def test_lt_gemm_strided_out_and_operands():
    torch.manual_seed(1)
    M, N, K = 192, 160, 256
    big_a = torch.randn(K, M + 64, device=DEV).bfloat16()
    a = big_a[:, :M]  # row stride M + 64
    b = torch.randn(K, N, device=DEV).bfloat16()
    bucket = torch.full((M, N + 32), 7.0, device=DEV)
    out = bucket[:, 16:16 + N]  # a view into a larger buffer, like a DDP bucket slot
    ops().lt_gemm_out(a, b, True, False, out)
    torch.testing.assert_close(out, _ref(a, b, True, False), rtol=1e-3, atol=1e-2)
    assert torch.all(bucket[:, :16] == 7.0) and torch.all(bucket[:, 16 + N:] == 7.0)


def test_lt_gemm_table_records_tuned_problems():
    a = torch.randn(512, 256, device=DEV).bfloat16()
    b = torch.randn(512, 128, device=DEV).bfloat16()
    ops().lt_gemm(a, b, True, False, torch.float32)
    tab = list(ops().lt_gemm_table())
    rows = [tab[i:i + 10] for i in range(0, len(tab), 10)]
    hit = [r for r in rows if r[:6] == [256, 128, 512, 1, 0, 0]]
    assert hit and hit[0][6] >= 1 and 0 <= hit[0][7] < hit[0][6] and hit[0][8] > 0


def test_lt_gemm_shape_checks():
    a = torch.randn(64, 32, device=DEV).bfloat16()
    with pytest.raises(RuntimeError):
        ops().lt_gemm(a, torch.randn(48, 16, device=DEV).bfloat16(), False, False, torch.float32)
    with pytest.raises(RuntimeError):
        ops().lt_gemm(a.float(), torch.randn(32, 16, device=DEV), False, False, torch.float32)


def test_model_step_with_lt_gemm_matches_blas(monkeypatch):
    from cs336_systems import ops as cops
    from cs336_systems.models import BasicsTransformerLM
    from cs336_systems.ops import gemm

    torch.manual_seed(0)
    model = BasicsTransformerLM(vocab_size=512, context_length=128, d_model=256, num_layers=2, num_heads=4, d_ff=1024, device=DEV)
    x = torch.randint(0, 512, (4, 128), device=DEV)
    y = torch.randint(0, 512, (4, 128), device=DEV)

    def run():
        model.zero_grad(set_to_none=True)
        with torch.autocast("cuda", dtype=torch.bfloat16):
            logits = model(x)
            loss = cops.cross_entropy(logits, y)
        loss.backward()
        return logits.float(), {n: p.grad.clone() for n, p in model.named_parameters()}

    monkeypatch.setenv("CS336_GEMM", "blas")
    l_ref, g_ref = run()
    monkeypatch.setenv("CS336_GEMM", "lt")
    assert gemm.lt_gemm_enabled()
    calls = []
    real = ops()

    class Spy:
        def __getattr__(self, name):
            fn = getattr(real, name)
            if name.startswith("lt_gemm"):
                return lambda *a: (calls.append(name), fn(*a))[1]
            return fn

    monkeypatch.setattr(gemm, "ops", lambda: Spy())
    l_lt, g_lt = run()
    assert "lt_gemm" in calls and "lt_gemm_out" in calls or calls.count("lt_gemm") >= 3
    torch.testing.assert_close(l_lt, l_ref, rtol=2e-2, atol=2e-2)
    for n in g_ref:
        scale = g_ref[n].abs().max().item() + 1e-6
        torch.testing.assert_close(g_lt[n] / scale, g_ref[n] / scale, rtol=0, atol=2e-2, msg=n)


def test_best_mode_picks_per_problem_and_matches_fp32(monkeypatch):
    """CS336_GEMM=best: every projection-GEMM entry point returns the fp32-reference result whichever
    backend wins the timing, and the decision is cached once per problem."""
    from cs336_systems.ops import gemm

    monkeypatch.setenv("CS336_GEMM", "best")
    gemm._BEST.clear()
    torch.manual_seed(3)
    T, K, N = 512, 256, 384
    x = torch.randn(T, K, device=DEV).bfloat16()
    w = torch.randn(N, K, device=DEV).bfloat16()
    dy = torch.randn(T, N, device=DEV).bfloat16()
    y = gemm.mm_nt(x, w)
    torch.testing.assert_close(y.float(), x.float() @ w.float().t(), rtol=1e-2, atol=1e-2 * K**0.5 * 4)
    dx = gemm.mm_nn(dy, w)
    torch.testing.assert_close(dx.float(), dy.float() @ w.float(), rtol=1e-2, atol=1e-2 * N**0.5 * 4)
    ref_dw = dy.float().t() @ x.float()
    out = torch.zeros(N, K, device=DEV)
    assert gemm.mm_tn_fp32(dy, x, out=out) is out
    torch.testing.assert_close(out, ref_dw, rtol=1e-3, atol=1e-3 * ref_dw.abs().max().item())
    xt = x.t().contiguous()
    dw2 = gemm.mm_tn_fp32_xt(dy, xt)
    torch.testing.assert_close(dw2, ref_dw, rtol=1e-3, atol=1e-3 * ref_dw.abs().max().item())
    choices = gemm.gemm_choices()
    assert {k[0] for k in choices} == {"nt", "nn", "tn32", "tt32"}
    n = len(choices)
    gemm.mm_nt(x, w)
    assert len(gemm.gemm_choices()) == n  # cached, not re-timed


def test_best_mode_times_cs336_gemm_where_it_applies(monkeypatch):
    """At shapes the cs336 MFMA GEMM tiles (160/256 multiples, K % 64 == 0) `best` times it next to
    hipBLASLt's default and the autotuned lt_gemm, and any winner is numerically right."""
    from cs336_systems.ops import gemm

    monkeypatch.setenv("CS336_GEMM", "best")
    gemm._BEST.clear()
    gemm._BEST_TIMES.clear()
    torch.manual_seed(4)
    T, K, N = 2560, 1600, 1600  # XL o-projection widths at 2560 tokens
    x = torch.randn(T, K, device=DEV).bfloat16()
    w = torch.randn(N, K, device=DEV).bfloat16()
    dy = torch.randn(T, N, device=DEV).bfloat16()
    y = gemm.mm_nt(x, w)
    torch.testing.assert_close(y.float(), x.float() @ w.float().t(), rtol=1e-2, atol=1e-2 * K**0.5 * 4)
    dx = gemm.mm_nn(dy, w)
    torch.testing.assert_close(dx.float(), dy.float() @ w.float(), rtol=1e-2, atol=1e-2 * N**0.5 * 4)
    ref_dw = dy.float().t() @ x.float()
    dw = gemm.mm_tn_fp32(dy, x)
    torch.testing.assert_close(dw, ref_dw, rtol=1e-3, atol=1e-3 * ref_dw.abs().max().item())
    timed = gemm.gemm_timings()
    assert len(timed) == 3
    for key, times in timed.items():
        # fp32 weight gradients also time the split-K candidates (gemm._splitk_cands); NT problems
        # gemm8 tiles (M % 256, N % 320/256, K % 64) also time it ("g8")
        assert {"blas", "lt", "cs336"} <= set(times), (key, times)
        assert all(t in ("blas", "lt", "cs336") or (key[0] == "nt" and t == "g8") or (key[0] in ("tn32", "tt32", "dyt32n", "dyt32t") and t.startswith("splitk")) for t in times), (key, times)
        assert gemm.gemm_choices()[key] in times
