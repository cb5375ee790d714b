"""Reference-path module (``cs336_systems/flashattentioncode.py``): FA2 latency/TFLOPS sweeps with a
HIP-event do_bench; see :mod:`cs336_systems.bench.flash`."""

from .bench.flash import attn_flops, bench_one, leaderboard, main  # noqa: F401


def benchmark_FA(context_length: int, d: int, dtype: str = "bf16", causal: bool = True, batch: int = 1):
    """HIP FA2 vs naive PyTorch attention: fwd / bwd / fwd+bwd ms and TFLOPS (reference ``:15-67``)."""
    return [bench_one(impl, batch, 1, context_length, d, dtype, causal) for impl in ("hip_fa2", "torch_naive")]


if __name__ == "__main__":
    main()
