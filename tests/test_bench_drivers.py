"""The benchmark / training drivers run end to end on CPU (Gloo for the distributed ones)."""

import pytest

from cs336_systems.bench import attention, collectives, ddp, e2e, precision


@pytest.mark.parametrize("variant", ["naive", "flat", "individual", "bucketed"])
def test_ddp_driver_matches_single_process(variant):
    # --check asserts on every rank that the DP model tracks a single-process replica
    ddp.main(["--cpu", "--world-size", "2", "--size", "tiny", "--ctx", "32", "--batch", "4", "--steps", "2", "--warmup", "1", "--variant", variant, "--bucket-mb", "0.05", "--check"])


def test_ddp_driver_sharded():
    ddp.main(["--cpu", "--world-size", "2", "--size", "tiny", "--ctx", "32", "--batch", "4", "--steps", "2", "--warmup", "1", "--sharded", "--check"])


def test_collectives_cpu():
    collectives.main(["--cpu", "--world-size", "2", "--sizes-mb", "0.01", "0.1", "--iters", "2", "--warmup", "1", "--ops", "all_reduce", "all_gather", "reduce_scatter"])


def test_e2e_benchmark_cpu():
    r = e2e.run_simple_benchmark("tiny", 32, 2, warmup_steps=1, timed_steps=2, device="cpu")
    for k in ("fwd_ms", "bwd_ms", "opt_ms", "step_ms", "tokens_per_s"):
        assert r[k] > 0


def test_attention_benchmark_cpu():
    for impl in ("naive", "flash"):
        r = attention.compare_attention_methods(32, 16, impl, batch=2, iters=1, warmup=1, device="cpu")
        assert "error" not in r and r["fwd_ms"] > 0


def test_precision_demo():
    acc = precision.accumulation_demo()
    assert abs(acc["fp32 += fp32"] - 10) < 1e-3 and abs(acc["fp16 += fp16"] - 10) > 1e-2
    assert precision.autocast_dtypes(device="cpu")["parameters"] == "torch.float32"


@pytest.mark.parametrize(
    "name",
    ["benchmark", "benchmark_attention", "ddp_bucketed_overlapped_sharded", "ddp_overlap", "distributed_communication_single",
     "flash_attention", "flashattentioncode", "mixed_precision_testing", "naive_ddp", "precision", "transformer_annotated"],
)
def test_reference_module_paths_import(name):
    """Every module path of the reference's cs336_systems package exists here."""
    import importlib

    importlib.import_module(f"cs336_systems.{name}")


def test_ddp_overlap_name_is_working_overlapped_ddp():
    from cs336_systems.ddp_overlap import DDPOverlap
    from cs336_systems.parallel import DDPIndividual

    assert DDPOverlap is DDPIndividual


def test_reference_ddp_script_switches():
    """The reference script's switches (ddp_bucketed_overlapped_sharded.py:366-419) map onto the
    bench.ddp driver with the reference hyper-parameters; later options override them."""
    from cs336_systems.ddp_bucketed_overlapped_sharded import reference_argv

    def parsed(argv):
        return ddp.parse(reference_argv(argv))

    a = parsed([])
    assert (a.variant, a.world_size, a.size, a.ctx, a.batch, a.lr, a.wd, a.steps) == ("naive", 1, "small", 128, 128, 1e-3, 0.1, 50)
    assert (parsed(["--distributed"]).variant, parsed(["--ddp"]).variant) == ("naive", "individual")
    b = parsed(["--ddp_bucketed", "--sharded", "--size", "tiny"])
    assert (b.variant, b.sharded, b.world_size, b.size) == ("bucketed", True, 2, "tiny")
    assert not parsed(["--distributed", "--sharded"]).sharded  # the reference shards under its DDP wrappers only
    ddp.main(reference_argv(["--ddp_bucketed", "--sharded", "--cpu", "--size", "tiny", "--ctx", "32", "--batch", "4",
                             "--steps", "2", "--warmup", "1", "--check"]))
