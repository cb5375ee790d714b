"""Reference-path module (``cs336_systems/ddp_bucketed_overlapped_sharded.py``): DDP,
DDP_Bucketed and ShardedStateOptimizer, backed by ``cs336_systems.parallel``. The training driver
of that file lives in ``cs336_systems.bench.ddp`` (``python -m cs336_systems.bench.ddp``)."""

from .parallel.ddp import DDP, DDP_Bucketed, DDPBucketed, DDPIndividual, FlatDDP, NaiveDDP  # noqa: F401
from .parallel.sharded_optimizer import ShardedOptimizer, ShardedStateOptimizer  # noqa: F401
