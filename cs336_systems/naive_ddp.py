"""Reference-path module (``cs336_systems/naive_ddp.py``): naive (per-parameter) and flat
data-parallel training; see :mod:`cs336_systems.bench.ddp` and :mod:`cs336_systems.parallel.ddp`."""

from .bench.ddp import main, parse, train_ddp as _train  # noqa: F401
from .parallel.ddp import FlatDDP, NaiveDDP  # noqa: F401


def train_ddp(rank: int, world_size: int, argv: list[str] | None = None):
    """Naive per-parameter blocking all-reduce (reference ``:269-442``)."""
    return _train(rank, world_size, parse(["--variant", "naive", *(argv or [])]))


def train_ddp_flat(rank: int, world_size: int, argv: list[str] | None = None):
    """One all-reduce over all gradients (reference ``:444-634``)."""
    return _train(rank, world_size, parse(["--variant", "flat", *(argv or [])]))


if __name__ == "__main__":
    main()
