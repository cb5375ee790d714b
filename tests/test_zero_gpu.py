"""ZeRO-2 (parallel/zero.py) on the GPU path: a fused-layout LM under bf16 autocast with bf16
compute shadows, on a one-rank RCCL group, trains exactly like the plain fused AdamW (the shard is
the whole bucket; the shadows come from a cast after the param all-gather instead of the update
kernel), and a 2-rank rehearsal of bench.py --ddp zero on one GPU (gloo, host-staged collectives)."""

import json
import os
import subprocess
import sys

import pytest
import torch
import torch.distributed as dist

from cs336_systems import ops
from cs336_systems.models import BasicsTransformerLM
from cs336_systems.models.fused import get_shadow, shadow_valid
from cs336_systems.parallel.comm import find_free_port
from cs336_systems.parallel.zero import ZeroDDP

pytestmark = pytest.mark.gpu
DEV = "cuda"
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OPT = dict(lr=1e-3, betas=(0.9, 0.95), eps=1e-8, weight_decay=0.01)


@pytest.fixture(scope="module")
def rccl_world1():
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(find_free_port()))
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device(DEV, 0))
    yield
    dist.destroy_process_group()


def _lm():
    torch.manual_seed(0)
    return BasicsTransformerLM(vocab_size=512, context_length=128, d_model=256, num_layers=2, num_heads=4, d_ff=1024,
                               device=DEV, fused_layout=True)


@pytest.mark.parametrize("collectives,gather", [(False, "auto"), (True, "fp32"), (True, "bf16")])
def test_zero_world1_matches_fused_adamw(rccl_world1, collectives, gather):
    """collectives=True also runs the RCCL reduce-scatter and the in-place all-gather: of the fp32
    masters + a shadow cast (gather fp32), or of the bf16 shadows the update kernel wrote, with the
    fp32 masters gathered on demand by state_dict() (gather bf16)."""
    ref = _lm()
    ref_opt = ops.FusedAdamW(ref.parameters(), bf16_shadows=True, **OPT)
    zero = ZeroDDP(_lm(), bucket_size_mb=2.0, bf16_shadows=True, gather_dtype=gather,
                   _collectives_at_world1=collectives, **OPT)
    assert len(zero.buckets) > 2
    kinds = {b["gather"] for b in zero.bucket_summary()}
    assert kinds == ({"bf16", "fp32"} if gather == "bf16" else {"fp32"})
    opt = zero.optimizer
    for it in range(3):
        x = torch.randint(0, 512, (4, 128), device=DEV, generator=torch.Generator(DEV).manual_seed(it))
        losses = []
        for model, o, z in ((ref, ref_opt, None), (zero, opt, zero)):
            o.zero_grad(set_to_none=True)
            with torch.autocast("cuda", dtype=torch.bfloat16):
                loss = ops.cross_entropy(model(x), x)
            loss.backward()
            if z is not None:
                z.finish_gradient_synchronization()
            o.step()
            losses.append(loss.detach().float())
        torch.testing.assert_close(losses[1], losses[0], rtol=1e-5, atol=1e-5)
        sd = zero.state_dict()
        for (n, a), b in zip(sd.items(), ref.state_dict().values()):
            torch.testing.assert_close(a, b, rtol=1e-5, atol=1e-6, msg=lambda m, n=n: f"{n}: {m}")
    # after the forward pre-hooks ran, every 2-D weight reads a valid shadow equal to its bf16 cast
    with torch.autocast("cuda", dtype=torch.bfloat16):
        zero(x)
    for p in zero.module.parameters():
        if p.dim() == 2:
            assert shadow_valid(p)
            assert torch.equal(get_shadow(p), p.detach().bfloat16())


def test_zero_bench_two_ranks_one_gpu():
    env = dict(os.environ, CS336_DIST_BACKEND="gloo", HSA_ENABLE_IPC_MODE_LEGACY="0")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2", "--master-addr",
           "127.0.0.1", "--master-port", str(find_free_port()), os.path.join(ROOT, "bench.py"), "--gpus", "2", "--model",
           "small", "--ctx", "128", "--batch", "4", "--steps", "2", "--warmup", "1", "--ddp", "zero", "--bucket-mb", "64"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=240, env=env, cwd=ROOT)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    line = [ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1]
    out = json.loads(line)
    assert out["n_gpus"] == 2 and out["config"]["parallelism"] == "dp2+zero2"
    assert out["final_loss"] == out["final_loss"] and out["final_loss"] < 20  # finite, trained


def _step(model, opt, z, x):
    opt.zero_grad(set_to_none=True)
    with torch.autocast("cuda", dtype=torch.bfloat16):
        loss = ops.cross_entropy(model(x), x)
    loss.backward()
    if z is not None:
        z.finish_gradient_synchronization()
    opt.step()


@pytest.mark.parametrize("gather", ["fp32", "bf16"])
def test_zero_gather_keeps_wt_shadows(rccl_world1, gather):
    """after the parameter all-gather the Wᵀ shadows are re-written (one transpose
    per fused group), so the forward uses Wᵀ for every projection instead of transposing."""
    from cs336_systems.models.fused import get_shadow_t, shadow_t_valid

    zero = ZeroDDP(_lm(), bucket_size_mb=2.0, bf16_shadows=True, gather_dtype=gather, _collectives_at_world1=True, **OPT)
    x = torch.randint(0, 512, (4, 128), device=DEV, generator=torch.Generator(DEV).manual_seed(0))
    _step(zero, zero.optimizer, zero, x)
    with torch.autocast("cuda", dtype=torch.bfloat16):
        zero(x)  # forward pre-hooks wait for the gathers and refresh shadows + Wᵀ
    n = 0
    for name, p in zero.module.named_parameters():
        if p.dim() == 2 and get_shadow_t(p) is not None:
            assert shadow_t_valid(p), name
            assert torch.equal(get_shadow_t(p), get_shadow(p).t()), name
            n += 1
    assert n >= 4 * 2  # q/k/v/o/w1/w2/w3 of both layers (+ lm head)


def test_zero_fp32_forward_after_bf16_gather(rccl_world1):
    """with gather_dtype='auto'/'bf16' only the bf16 shadows travel; a forward that reads
    the fp32 masters (no autocast) must gather them first, and match the unsharded model."""
    ref = _lm()
    ref_opt = ops.FusedAdamW(ref.parameters(), bf16_shadows=True, **OPT)
    zero = ZeroDDP(_lm(), bucket_size_mb=2.0, bf16_shadows=True, gather_dtype="bf16", _collectives_at_world1=True, **OPT)
    x = torch.randint(0, 512, (4, 128), device=DEV, generator=torch.Generator(DEV).manual_seed(1))
    for model, o, z in ((ref, ref_opt, None), (zero, zero.optimizer, zero)):
        _step(model, o, z, x)
    assert zero._masters_stale
    with torch.no_grad():
        got = zero(x).float()
        want = ref(x).float()
    assert not zero._masters_stale
    torch.testing.assert_close(got, want, rtol=1e-4, atol=1e-4)
