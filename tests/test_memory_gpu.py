"""Forward-only memory profile is a grad-mode forward (the round-1 forward rows
were no_grad measurements). The forward peak minus the model's own allocations must exceed a
lower bound of the activations a grad-mode forward has to keep (per layer: the QKV input, the
rotated q|k, the W1|W3 output and the gate output), and a no_grad forward of the same model stays
far below it."""

import pytest
import torch

pytestmark = pytest.mark.gpu


def test_forward_memory_profile_keeps_activations():
    from cs336_systems.bench.e2e import run_memory_profile
    from cs336_systems.models import build_model, get_model_config

    if not torch.cuda.is_available():
        pytest.skip("needs a GPU")
    size, ctx, B = "small", 256, 4
    cfg = get_model_config(size)
    L, d, dff = cfg["num_layers"], cfg["d_model"], cfg["d_ff"]
    dev = torch.device("cuda")
    torch.cuda.empty_cache()
    torch.cuda.reset_peak_memory_stats(dev)
    base = torch.cuda.memory_allocated(dev)
    peak = run_memory_profile(size, ctx, mode="forward", mixed_precision=False, batch_size=B) * 2**20
    m = build_model(size, ctx, device=dev)
    model_bytes = sum(p.numel() * p.element_size() for p in m.parameters())
    del m
    # fp32 forward: per layer at least d (QKV input) + 2d (rotated q|k) + 2 d_ff (W1|W3 out) + d_ff (gate)
    bound = L * B * ctx * (3 * d + 3 * dff) * 4
    act = peak - base - model_bytes
    assert act > 0.8 * bound, f"forward keeps {act / 2**20:.0f} MiB of activations, bound {bound / 2**20:.0f} MiB"
    # a no_grad forward keeps none of them
    torch.cuda.empty_cache()
    torch.cuda.reset_peak_memory_stats(dev)
    m = build_model(size, ctx, device=dev)
    base2 = torch.cuda.memory_allocated(dev)
    with torch.no_grad():
        m(torch.randint(0, 10000, (B, ctx), device=dev))
    torch.cuda.synchronize()
    assert torch.cuda.max_memory_allocated(dev) - base2 < 0.5 * bound
