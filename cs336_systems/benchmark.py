"""Reference-path module (``cs336_systems/benchmark.py``): end-to-end timing and memory profiling.
Implementation: :mod:`cs336_systems.bench.e2e` (``python -m cs336_systems.benchmark`` works too)."""

from .bench.e2e import main, run_memory_profile, run_simple_benchmark  # noqa: F401
from .models.configs import MODEL_CONFIGS, get_model_config  # noqa: F401

run_memory_foward_fullstep = run_memory_profile  # reference spelling


def run_all_benchmarks(sizes=("small", "medium", "large", "xl", "2.7b"), context_length=256, batch_size=4, mixed_precision=False, compile_options=(False, True)):
    """Sweep sizes x compile (the reference dropped the compile flag; here it is forwarded)."""
    rows = []
    for size in sizes:
        for c in compile_options:
            rows.append(run_simple_benchmark(size, context_length, batch_size, 2, 10, mixed_precision, c))
    return rows


if __name__ == "__main__":
    main()
