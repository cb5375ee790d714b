"""Fused SwiGLU FFN (models/fused.py SwiGLUFFNFn: gate in the gemm8 epilogues) against the unfused
module path (GEMMs + separate HIP gate kernels) and an fp32 PyTorch reference, forward and all
gradients, under bf16 autocast with the bf16/Wᵀ shadows the training step uses."""

import pytest
import torch

pytestmark = pytest.mark.gpu


def _setup(d_model=320, d_ff=640, tokens=512, seed=0):
    from cs336_systems import ops
    from cs336_systems.models.transformer import SwiGLU

    if not torch.cuda.is_available():
        pytest.skip("needs a GPU")
    assert ops.load_ext(), ops.load_error()
    torch.manual_seed(seed)
    m = SwiGLU(d_model, d_ff, device="cuda")
    m.group_()
    x = torch.randn(2, tokens // 2, d_model, device="cuda")
    dy = torch.randn(2, tokens // 2, d_model, device="cuda")
    return m, x, dy


def _run(m, x, dy, fused: bool, monkeypatch):
    monkeypatch.setenv("CS336_SWIGLU_FUSED", "1" if fused else "0")
    for p in m.parameters():
        p.grad = None
    xx = x.clone().requires_grad_(True)
    with torch.autocast("cuda", dtype=torch.bfloat16):
        out = m(xx)
    out.backward(dy)
    return out.float(), xx.grad.float(), [p.grad.float().clone() for p in (m.w1.weight, m.w3.weight, m.w2.weight)]


def _rel(a, b):
    return float((a - b).norm() / b.norm().clamp_min(1e-30))


@pytest.mark.parametrize("d_model,d_ff", [(320, 640), (256, 512), (1600, 6400)])
def test_fused_ffn_matches_unfused_and_fp32(monkeypatch, d_model, d_ff):
    from cs336_systems.models.fused import attach_bf16_shadows

    m, x, dy = _setup(d_model, d_ff, tokens=512 if d_model < 1600 else 1024)
    attach_bf16_shadows(m)  # bf16 + Wᵀ shadows, as FusedAdamW keeps them in training
    of, dxf, gf = _run(m, x, dy, True, monkeypatch)
    ou, dxu, gu = _run(m, x, dy, False, monkeypatch)
    # fp32 reference
    w1, w3, w2 = (p.detach().float() for p in (m.w1.weight, m.w3.weight, m.w2.weight))
    xr = x.clone().requires_grad_(True)
    w1r, w3r, w2r = (w.clone().requires_grad_(True) for w in (w1, w3, w2))
    a, b = xr @ w1r.t(), xr @ w3r.t()
    ref = (torch.nn.functional.silu(a) * b) @ w2r.t()
    ref.backward(dy)
    for got, unf, r, name in ((of, ou, ref.detach(), "out"), (dxf, dxu, xr.grad, "dx"),
                              (gf[0], gu[0], w1r.grad, "dw1"), (gf[1], gu[1], w3r.grad, "dw3"),
                              (gf[2], gu[2], w2r.grad, "dw2")):
        assert _rel(got, r) < 2e-2, (name, _rel(got, r), _rel(unf, r))
        assert _rel(got, unf) < 2e-2, (name, _rel(got, unf))


def test_fused_ffn_retain_graph_and_version_check(monkeypatch):
    """The stages' saved tensors go through the Function's save_for_backward: a
    retain_graph second backward gives the same gradients, and a saved weight rewritten in place
    before backward is caught by autograd's version counter instead of used silently."""
    from cs336_systems.models.fused import attach_bf16_shadows, get_shadow_t

    m, x, dy = _setup(320, 640)
    attach_bf16_shadows(m)
    monkeypatch.setenv("CS336_SWIGLU_FUSED", "1")
    xx = x.clone().requires_grad_(True)
    with torch.autocast("cuda", dtype=torch.bfloat16):
        out = m(xx)
    out.backward(dy, retain_graph=True)
    g1 = [p.grad.clone() for p in (m.w1.weight, m.w3.weight, m.w2.weight)] + [xx.grad.clone()]
    for p in m.parameters():
        p.grad = None
    xx.grad = None
    out.backward(dy)
    g2 = [p.grad for p in (m.w1.weight, m.w3.weight, m.w2.weight)] + [xx.grad]
    for a, b in zip(g1, g2):
        torch.testing.assert_close(a, b, rtol=0, atol=0)
    # a saved Wᵀ shadow bumped in place between forward and backward
    with torch.autocast("cuda", dtype=torch.bfloat16):
        out = m(x.clone().requires_grad_(True))
    wt = get_shadow_t(m.w2.weight)
    assert wt is not None
    wt.add_(0)
    with pytest.raises(RuntimeError, match="modified by an inplace operation"):
        out.backward(dy)


def test_fused_ffn_backward_frees_each_layers_h(monkeypatch):
    """Once a layer's backward ran, nothing of its forward (h, y, X) may stay alive for the rest of the
    backward: with n layers chained, the memory held when the FIRST layer's input gradient arrives
    must not grow with n beyond the weight gradients (a forward-only closure on the stage once kept
    every layer's h: +30 GB on the XL step)."""
    from cs336_systems.models.fused import attach_bf16_shadows
    from cs336_systems.models.transformer import SwiGLU

    monkeypatch.setenv("CS336_SWIGLU_FUSED", "1")
    d_model, d_ff, tokens = 320, 1280, 4096

    def held_at_first_grad(n):
        torch.manual_seed(0)
        layers = [SwiGLU(d_model, d_ff, device="cuda") for _ in range(n)]
        for m in layers:
            m.group_()
            attach_bf16_shadows(m)
        x = torch.randn(1, tokens, d_model, device="cuda", requires_grad=True)
        seen = {}
        torch.cuda.synchronize()
        base = torch.cuda.memory_allocated()
        with torch.autocast("cuda", dtype=torch.bfloat16):
            hcur = x * 1.0
            def hook(g):
                seen.setdefault("mem", torch.cuda.memory_allocated())

            hcur.register_hook(hook)
            for m in layers:
                hcur = m(hcur)
        hcur.float().sum().backward()
        grads = sum(p.grad.numel() * 4 for m in layers for p in m.parameters())
        return seen["mem"] - base - grads

    h_bytes = tokens * d_ff * 2
    grow = held_at_first_grad(6) - held_at_first_grad(2)
    assert grow < h_bytes, f"memory held at the first layer's grad grew by {grow / 2**20:.1f} MiB for 4 more layers"
