"""RCCL path on the 1-GPU box: every DP variant (and ZeRO-1) with world_size 1 over the nccl(=RCCL)
backend, bf16 autocast, fused layout (dW GEMMs writing into the DDP buckets), checked step by step
against an unwrapped replica. Multi-rank RCCL runs happen in the driver's 8-GPU scaling bench."""

import pytest

from cs336_systems.bench import ddp

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("variant", ["naive", "flat", "individual", "bucketed"])
def test_ddp_variants_rccl_world1(variant):
    ddp.main(["--world-size", "1", "--size", "tiny", "--ctx", "64", "--batch", "4", "--steps", "3", "--warmup", "1", "--variant", variant, "--bucket-mb", "1", "--check"])


@pytest.mark.parametrize("variant", ["individual", "bucketed"])
@pytest.mark.parametrize("sharded", [False, True])
def test_ddp_two_ranks_one_gpu_gloo(variant, sharded):
    """2 ranks sharing cuda:0 (gloo over GPU tensors): the real multi-rank path on GPU kernels —
    dW written into buckets from the side stream, all-reduce after the stream sync, ZeRO-1
    all-gather + shadow re-cast — against a single-process replica trained on the global batch."""
    args = ["--world-size", "2", "--gloo-gpu", "--size", "tiny", "--ctx", "64", "--batch", "4", "--steps", "3",
            "--warmup", "1", "--variant", variant, "--bucket-mb", "1", "--check"]
    ddp.main(args + (["--sharded"] if sharded else []))


def test_sharded_rccl_world1():
    ddp.main(["--world-size", "1", "--size", "tiny", "--ctx", "64", "--batch", "4", "--steps", "3", "--warmup", "1", "--sharded", "--check"])
