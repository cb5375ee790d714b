"""Fused AdamW that also writes the transposed bf16 shadow Wᵀ (csrc/ops/multi_tensor.hip
adamw_t_kernel): bitwise the same update as the 1-D kernel, Wᵀ bitwise equal to
the transpose of the bf16 shadow, column-block views of grouped Wᵀ, and a model step in which the
forward uses those Wᵀ instead of transposing (no transpose16 launches for weights)."""

import pytest
import torch

from cs336_systems import ops
from cs336_systems.models import BasicsTransformerLM
from cs336_systems.models.fused import compute_weight_t, get_shadow, get_shadow_t, shadow_t_valid

pytestmark = pytest.mark.gpu
DEV = "cuda"
OPT = dict(lr=1e-2, betas=(0.9, 0.95), eps=1e-8, weight_decay=0.1)


@pytest.mark.parametrize("shape", [(1600, 1600), (10000, 1600), (1600, 6400), (264, 72)])
@pytest.mark.parametrize("gdt", [torch.float32, torch.bfloat16])
def test_adamw_t_matches_adamw(shape, gdt):
    assert ops.load_ext(), ops.load_error()
    torch.manual_seed(0)
    p = torch.randn(*shape, device=DEV)
    g = torch.randn(*shape, device=DEV).to(gdt)
    m = torch.randn(*shape, device=DEV).abs() * 1e-2
    v = torch.randn(*shape, device=DEV).abs() * 1e-3
    # Wᵀ as a column block of a wider (C, R + 40) tensor, like one weight of a grouped Wᵀ
    wt_base = torch.zeros(shape[1], shape[0] + 40, device=DEV, dtype=torch.bfloat16)
    wt = wt_base[:, 8 : 8 + shape[0]]
    ref = [t.clone() for t in (p, m, v)]
    sh, sh_ref = torch.empty_like(p, dtype=torch.bfloat16), torch.empty_like(p, dtype=torch.bfloat16)
    for step in (1, 2, 3):
        torch.ops.cs336.adamw_step([ref[0]], [g], [ref[1]], [ref[2]], [sh_ref], 1e-2, 0.9, 0.95, 1e-8, 0.1, step)
        torch.ops.cs336.adamw_step_t([p], [g], [m], [v], [sh], [wt], 1e-2, 0.9, 0.95, 1e-8, 0.1, step)
    torch.cuda.synchronize()
    for a, b in zip((p, m, v, sh), (*ref, sh_ref)):
        assert torch.equal(a, b)
    assert torch.equal(wt, sh.t())
    assert torch.count_nonzero(wt_base[:, :8]) == 0 and torch.count_nonzero(wt_base[:, 8 + shape[0]:]) == 0


def _lm():
    torch.manual_seed(0)
    return BasicsTransformerLM(vocab_size=512, context_length=128, d_model=256, num_layers=2, num_heads=4, d_ff=1024,
                               device=DEV, fused_layout=True)


def test_model_step_uses_adamw_written_wt():
    model = _lm()
    opt = ops.FusedAdamW(model.parameters(), bf16_shadows=True, **OPT)
    att = model.layers[0].attn
    qkv = [att.q_proj.weight, att.k_proj.weight, att.v_proj.weight]
    x = torch.randint(0, 512, (4, 128), device=DEV)
    for _ in range(2):
        opt.zero_grad(set_to_none=True)
        with torch.autocast("cuda", dtype=torch.bfloat16):
            loss = ops.cross_entropy(model(x), x)
        loss.backward()
        opt.step()
    torch.cuda.synchronize()
    for p in model.parameters():
        if p.dim() == 2 and get_shadow_t(p) is not None:
            assert shadow_t_valid(p), "the update must leave Wᵀ valid"
            assert torch.equal(get_shadow_t(p), get_shadow(p).t())
            assert torch.equal(get_shadow(p), p.detach().bfloat16())
    wt = compute_weight_t(qkv)  # the grouped QKV Wᵀ is one strided view
    assert wt is not None and wt.shape == (256, 3 * 256)
    # an out-of-band master change invalidates the shadows and Wᵀ
    with torch.no_grad():
        att.q_proj.weight.mul_(1.0)
    assert not shadow_t_valid(att.q_proj.weight) and compute_weight_t(qkv) is None


def test_wt_path_matches_transpose_path(monkeypatch):
    """Training with the AdamW-written Wᵀ gives the same losses/weights as re-transposing."""
    a, b = _lm(), _lm()
    oa = ops.FusedAdamW(a.parameters(), bf16_shadows=True, **OPT)
    import cs336_systems.models.fused as fused

    ob = ops.FusedAdamW(b.parameters(), bf16_shadows=True, **OPT)
    for p in b.parameters():  # drop b's Wᵀ: its forward transposes every weight
        if hasattr(p, fused._SHADOW_T):
            delattr(p, fused._SHADOW_T)
    for it in range(3):
        x = torch.randint(0, 512, (4, 128), device=DEV, generator=torch.Generator(DEV).manual_seed(it))
        ls = []
        for m, o in ((a, oa), (b, ob)):
            o.zero_grad(set_to_none=True)
            with torch.autocast("cuda", dtype=torch.bfloat16):
                loss = ops.cross_entropy(m(x), x)
            loss.backward()
            o.step()
            ls.append(loss.item())
        assert ls[0] == ls[1]
    for pa, pb in zip(a.parameters(), b.parameters()):
        assert torch.equal(pa, pb)
