"""Reference-path module (``cs336_systems/distributed_communication_single.py``): all-reduce
microbenchmark; see :mod:`cs336_systems.bench.collectives`."""

from .bench.collectives import main, run_collective  # noqa: F401


def benchmark_allreduce(data_size_mb: float, device, warmup: int = 5, iters: int = 20) -> float:
    """Mean seconds of a blocking all-reduce of ``data_size_mb`` fp32 on this rank (process group
    must be initialised)."""
    import torch

    return run_collective("all_reduce", int(data_size_mb * 2**20), torch.device(device), warmup, iters)


if __name__ == "__main__":
    main()
