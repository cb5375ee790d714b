"""Reference-path module (``cs336_systems/benchmark_attention.py``); see :mod:`cs336_systems.bench.attention`."""

from .bench.attention import Attention, benchmark_attention, compare_attention_methods, main  # noqa: F401

if __name__ == "__main__":
    main()
