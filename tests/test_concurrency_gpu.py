"""GEMMs sharing the chip with other work (root cause of the round-1 concurrent-GEMM hang).

hipBLASLt's default solutions for the projection GEMMs are stream-K Tensile kernels ("SK3"): at
most one workgroup per CU, and the owner of a split tile spins on a flag that a later-dispatched
workgroup of the same grid sets (profiles/r2_streamk_hang.md). Two of them on two streams can
deadlock; one of them beside a *bounded* occupant (an RCCL kernel waits for its peers, which do
arrive) only waits. These tests pin both halves of that:

* the XL backward GEMM sequence (default hipBLASLt picks) completes beside a CU-occupying spin kernel
  on another stream that leaves no room for a GEMM workgroup on any CU, or holds half the CUs
  (the RCCL stand-in), with results bitwise equal to the serial run;
* hipBLASLt offers only stream-K solutions for these GEMMs, so the weight-gradient GEMMs the dW side
  stream issues run the cs336 MFMA GEMM (whole tiles per workgroup, no inter-workgroup waits), and
  two streams of those beside the main stream's stream-K GEMMs complete with identical results.
"""

import pytest
import torch

pytestmark = pytest.mark.gpu

T, D, F = 12288, 1600, 6400  # XL step: tokens per GPU, d_model, d_ff


def _ops():
    from cs336_systems import ops

    if not torch.cuda.is_available():
        pytest.skip("needs a GPU")
    assert ops.load_ext(), ops.load_error()
    return torch.ops.cs336


def _xl_layer_tensors(seed=0):
    g = torch.Generator(device="cuda").manual_seed(seed)
    r = lambda *s: (torch.randn(*s, device="cuda", generator=g) * 0.05).to(torch.bfloat16)  # noqa: E731
    return dict(
        x=r(T, D), h=r(T, F), dy_o=r(T, D), dy_13=r(T, 2 * F), dy_qkv=r(T, 3 * D),
        w_o=r(D, D), w_2=r(D, F), w_13=r(2 * F, D), w_qkv=r(3 * D, D),
    )


def _backward_gemms(t):
    """One XL layer's backward GEMMs in the step's orientations (dX bf16, dW fp32)."""
    out = []
    out.append(t["dy_o"] @ t["w_2"])  # W2 dX: (T, F)
    out.append(torch.mm(t["dy_o"].t(), t["h"], out_dtype=torch.float32))  # W2 dW
    out.append(t["dy_13"] @ t["w_13"])  # W1|W3 dX
    out.append(torch.mm(t["dy_13"].t(), t["x"], out_dtype=torch.float32))  # W1|W3 dW
    out.append(t["dy_o"] @ t["w_o"])  # O dX
    out.append(torch.mm(t["dy_o"].t(), t["x"], out_dtype=torch.float32))  # O dW
    out.append(t["dy_qkv"] @ t["w_qkv"])  # QKV dX
    out.append(torch.mm(t["dy_qkv"].t(), t["x"], out_dtype=torch.float32))  # QKV dW
    return out


def test_stream_k_mode_parser():
    cs = _ops()
    assert cs.tensile_stream_k_mode("Cijk_Alik_Bljk_BBS_MT160x256x64_SS1_SK3_SKFTR0_SKXCCM8_TLDS1_WG32_8_1") == 3
    assert cs.tensile_stream_k_mode("Cijk_Ailk_Bjlk_BSS_MT256x256x64_SK0_SKXCCM0_WG32_8_1") == 0
    assert cs.tensile_stream_k_mode("Cijk_Ailk_Bjlk_MT128x128x64_SKXCCM8_WG32") == 0


def test_hipblaslt_gemms_are_stream_k():
    """Pins the root cause: hipBLASLt's picks for the XL weight gradients are stream-K, and it offers
    no data-parallel solution for them on gfx950 (so the dW side stream cannot use hipBLASLt)."""
    cs = _ops()
    t = _xl_layer_tensors()
    for dy, x in ((t["dy_o"], t["h"]), (t["dy_13"], t["x"]), (t["dy_o"], t["x"]), (t["dy_qkv"], t["x"])):
        out = torch.empty(dy.shape[1], x.shape[1], device="cuda", dtype=torch.float32)
        name = cs.lt_gemm_kernel(dy, x, True, False, out, 0)
        assert cs.tensile_stream_k_mode(name) > 0, name
        with pytest.raises(RuntimeError, match="data-parallel"):
            cs.lt_gemm_kernel(dy, x, True, False, out, 1)


def test_side_stream_weight_gradients_use_cs336_gemm():
    """Every XL projection weight gradient except the Xᵀ-layout W1|W3 one and the lm_head (10000
    rows) is taken by the cs336 GEMM, which the dW side stream uses, and matches hipBLASLt."""
    _ops()
    from cs336_systems.ops import gemm

    t = _xl_layer_tensors()
    for dy, x in ((t["dy_o"], t["h"]), (t["dy_13"], t["x"]), (t["dy_o"], t["x"]), (t["dy_qkv"], t["x"])):
        assert gemm.dw_concurrent_ok(dy, x, False)
        assert not gemm.dw_concurrent_ok(dy, x.t().contiguous(), True)
        got = gemm.mm_tn_fp32(dy, x, concurrent_safe=True)
        ref = torch.mm(dy.t(), x, out_dtype=torch.float32)
        torch.testing.assert_close(got, ref, rtol=2e-3, atol=2e-3)
    lm = torch.randn(T, 10000, device="cuda").bfloat16()
    assert not gemm.dw_concurrent_ok(lm, t["x"], False)


@pytest.mark.parametrize("occupant", ["all_cus_no_room", "half_the_cus"])
def test_xl_backward_gemms_beside_occupying_kernel(occupant):
    cs = _ops()
    t = _xl_layer_tensors()
    ref = _backward_gemms(t)
    torch.cuda.synchronize()
    n_cu = torch.cuda.get_device_properties(0).multi_processor_count
    # no room: 64 KB per CU leaves < 124 KB (a stream-K GEMM workgroup) on every CU
    n_wg, lds = (n_cu, 64 * 1024) if occupant == "all_cus_no_room" else (n_cu // 2, 150 * 1024)
    counter = torch.zeros(1, dtype=torch.int32, device="cuda")
    side = torch.cuda.Stream()
    main = torch.cuda.current_stream()
    side.wait_stream(main)
    with torch.cuda.stream(side):
        cs.occupy(n_wg, lds, 50.0, counter)  # 50 ms, then exits
    got = _backward_gemms(t)  # main stream, default (stream-K) hipBLASLt solutions
    torch.cuda.synchronize()
    assert int(counter.item()) == n_wg
    for a, b in zip(got, ref):
        assert torch.equal(a, b)


def test_two_dw_streams_beside_stream_k_gemms():
    """Main stream: stream-K dX GEMMs; two side streams: cs336-GEMM weight gradients (the dW side
    stream's choice), plus a bounded occupant. Everything completes; dW matches the serial run."""
    cs = _ops()
    from cs336_systems.ops import gemm

    t = _xl_layer_tensors(1)
    pairs = [(t["dy_o"], t["h"]), (t["dy_13"], t["x"]), (t["dy_o"], t["x"]), (t["dy_qkv"], t["x"])]
    ref = [gemm.mm_tn_fp32(dy, x, concurrent_safe=True) for dy, x in pairs]
    torch.cuda.synchronize()
    main = torch.cuda.current_stream()
    s1, s2, s3 = torch.cuda.Stream(), torch.cuda.Stream(), torch.cuda.Stream()
    for s in (s1, s2, s3):
        s.wait_stream(main)
    counter = torch.zeros(1, dtype=torch.int32, device="cuda")
    with torch.cuda.stream(s3):
        cs.occupy(64, 32 * 1024, 20.0, counter)
    outs = []
    for i, (dy, x) in enumerate(pairs * 2):
        with torch.cuda.stream(s1 if i % 2 == 0 else s2):
            outs.append(gemm.mm_tn_fp32(dy, x, concurrent_safe=True))
    dx = [t["dy_13"] @ t["w_13"] for _ in range(3)]  # main stream, stream-K
    torch.cuda.synchronize()
    assert int(counter.item()) == 64
    for i, o in enumerate(outs):
        assert torch.equal(o, ref[i % len(pairs)])
    assert all(torch.equal(d, dx[0]) for d in dx)
