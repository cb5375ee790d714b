"""AdamW overlapped with backward (ops/adamw.py): parameters, optimizer state and bf16 shadows after
several steps are bitwise identical to the plain post-backward step, with and without the
weight-gradient side stream; a DDP world-1 (RCCL) run with per-bucket updates matches too."""

import pytest
import torch

from cs336_systems import ops
from cs336_systems.bench import ddp as ddp_bench
from cs336_systems.models import BasicsTransformerLM
from cs336_systems.models.fused import get_shadow

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _train(overlap, steps=3, chunk_mb=1.0):
    torch.manual_seed(0)
    model = BasicsTransformerLM(vocab_size=512, context_length=64, d_model=256, num_layers=3, num_heads=4, d_ff=768, device=DEV)
    opt = ops.FusedAdamW(model.parameters(), lr=1e-3, betas=(0.9, 0.95), weight_decay=0.1, bf16_shadows=True)
    if overlap:
        assert opt.enable_backward_overlap(chunk_mb=chunk_mb)
    g = torch.Generator(device=DEV).manual_seed(1)
    for _ in range(steps):
        x = torch.randint(0, 512, (4, 64), device=DEV, generator=g)
        opt.zero_grad(set_to_none=True)
        with torch.autocast("cuda", dtype=torch.bfloat16):
            loss = ops.cross_entropy(model(x), x)
        loss.backward()
        opt.step()
    torch.cuda.synchronize()
    return model, opt


@pytest.mark.parametrize("dw_stream", ["0", "1"])
def test_overlapped_step_is_bitwise_identical(monkeypatch, dw_stream):
    monkeypatch.setenv("CS336_DW_STREAM", dw_stream)
    ref, ref_opt = _train(False)
    got, got_opt = _train(True)
    assert got_opt.overlaps_backward and len(got_opt._ov.stepped) == 0
    for (n, a), b in zip(got.named_parameters(), ref.parameters()):
        torch.testing.assert_close(a, b, rtol=0, atol=0, msg=n)
        sa, sb = got_opt.state[a], ref_opt.state[b]
        assert sa["t"] == sb["t"]
        torch.testing.assert_close(sa["m"], sb["m"], rtol=0, atol=0, msg=n)
        torch.testing.assert_close(sa["v"], sb["v"], rtol=0, atol=0, msg=n)
        if get_shadow(a) is not None:
            torch.testing.assert_close(get_shadow(a), get_shadow(b), rtol=0, atol=0, msg=n)


def test_overlap_pause_falls_back_to_plain_step():
    model, opt = _train(True, steps=1)
    opt.set_backward_overlap(False)
    x = torch.randint(0, 512, (2, 64), device=DEV)
    opt.zero_grad(set_to_none=True)
    ops.cross_entropy(model(x), x).backward()
    assert not opt._ov.pending and not opt._ov.stepped
    opt.step()
    torch.cuda.synchronize()


def test_ddp_bucketed_overlap_rccl_world1():
    ddp_bench.main(["--world-size", "1", "--size", "tiny", "--ctx", "64", "--batch", "4", "--steps", "3", "--warmup", "1",
                    "--variant", "bucketed", "--bucket-mb", "1", "--overlap-opt", "--check"])
