"""Reference-path module (``cs336_systems/ddp_bucketed_overlapped_sharded.py``): DDP,
DDP_Bucketed and ShardedStateOptimizer, backed by ``cs336_systems.parallel``. The training driver
of that file lives in ``cs336_systems.bench.ddp`` (``python -m cs336_systems.bench.ddp``).

Run as a script it takes the reference's switches (``ddp_bucketed_overlapped_sharded.py:366-419``)
and its hyper-parameters (``:389-403``: the 768-wide 12-layer model, ctx 128, global batch 128,
lr 1e-3, weight decay 0.1, 50 steps, 2 ranks) and hands them to that driver:

    python -m cs336_systems.ddp_bucketed_overlapped_sharded [--distributed | --ddp | --ddp_bucketed] [--sharded]

``--distributed`` is the reference's hand-written per-parameter all-reduce (``naive``), ``--ddp``
its hook-overlapped per-parameter DDP (``individual``), ``--ddp_bucketed`` the bucketed one; no
switch trains one process. Any further ``bench.ddp`` option (``--size``, ``--steps``, ``--check``,
``--cpu``, ...) may follow and overrides the reference values.
"""

from .parallel.ddp import DDP, DDP_Bucketed, DDPBucketed, DDPIndividual, FlatDDP, NaiveDDP  # noqa: F401
from .parallel.sharded_optimizer import ShardedOptimizer, ShardedStateOptimizer  # noqa: F401

# reference hparams (:389-403) as bench.ddp options
REFERENCE_HPARAMS = ["--size", "small", "--ctx", "128", "--batch", "128", "--lr", "1e-3", "--wd", "0.1",
                     "--steps", "50"]


def reference_argv(argv: list[str] | None = None) -> list[str]:
    """Translate the reference's switches into ``cs336_systems.bench.ddp`` arguments."""
    import argparse

    ap = argparse.ArgumentParser(add_help=False)
    ap.add_argument("--distributed", action="store_true")
    ap.add_argument("--ddp", action="store_true")
    ap.add_argument("--ddp_bucketed", action="store_true")
    ap.add_argument("--sharded", action="store_true")
    a, rest = ap.parse_known_args(argv)
    if a.distributed:
        mode = ["--variant", "naive", "--world-size", "2"]
    elif a.ddp_bucketed:
        mode = ["--variant", "bucketed", "--world-size", "2"]
    elif a.ddp:
        mode = ["--variant", "individual", "--world-size", "2"]
    else:  # the reference's single-process training
        mode = ["--variant", "naive", "--world-size", "1"]
    if a.sharded and (a.ddp or a.ddp_bucketed):  # the reference shards only under its DDP wrappers
        mode.append("--sharded")
    return REFERENCE_HPARAMS + mode + rest


if __name__ == "__main__":
    import sys

    from .bench.ddp import main

    main(reference_argv(sys.argv[1:]))
