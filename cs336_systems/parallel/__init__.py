from .comm import (
    broadcast_module_,
    cleanup_distributed,
    default_backend,
    find_free_port,
    setup_distributed,
    spawn,
    supports_avg,
)
from .context_parallel import (
    RingAttention,
    disable_context_parallel,
    enable_context_parallel,
    ring_attention,
    sequence_positions,
    shard_sequence,
    ulysses_attention,
    unshard_sequence,
)
from .ddp import DDP, DDP_Bucketed, DDPBucketed, DDPIndividual, DEFAULT_BUCKET_MB, FlatDDP, NaiveDDP
from .sharded_optimizer import ShardedOptimizer, ShardedStateOptimizer
from .tensor_parallel import gather_tp_state_dict, tensor_parallel_
from .zero import ZeroDDP

DDP_VARIANTS = {
    "naive": NaiveDDP,
    "flat": FlatDDP,
    "individual": DDPIndividual,
    "bucketed": DDPBucketed,
}


def wrap_ddp(module, variant: str = "bucketed", bucket_size_mb: float | None = DEFAULT_BUCKET_MB, **kw):
    """Wrap ``module`` with one of the four DP variants by name."""
    cls = DDP_VARIANTS[variant]
    if cls is DDPBucketed:
        return cls(module, bucket_size_mb=bucket_size_mb, **kw)
    return cls(module, **kw)


__all__ = [
    "DDP",
    "DDP_Bucketed",
    "DDPBucketed",
    "DDPIndividual",
    "DDP_VARIANTS",
    "DEFAULT_BUCKET_MB",
    "RingAttention",
    "disable_context_parallel",
    "enable_context_parallel",
    "ring_attention",
    "sequence_positions",
    "shard_sequence",
    "unshard_sequence",
    "ulysses_attention",
    "FlatDDP",
    "NaiveDDP",
    "ShardedOptimizer",
    "ShardedStateOptimizer",
    "broadcast_module_",
    "cleanup_distributed",
    "default_backend",
    "find_free_port",
    "setup_distributed",
    "spawn",
    "supports_avg",
    "wrap_ddp",
    "ZeroDDP",
    "gather_tp_state_dict",
    "tensor_parallel_",
]
