"""Process-group setup and small collective helpers (RCCL on GPU, Gloo on CPU).

Reference parity: ``naive_ddp.py:35-51``, ``ddp_bucketed_overlapped_sharded.py:46-49``,
``distributed_communication_single.py:11-26`` and ``tests/common.py:71-94`` each hand-roll an
env:// rendezvous on localhost with ``mp.spawn``. Here one helper serves both launch styles:

* ``torchrun`` / ``python -m torch.distributed.run`` (``RANK``/``LOCAL_RANK``/``WORLD_SIZE`` in the
  env) — the way ``bench.py`` and the scaling runs are launched: one process per MI355X;
* ``mp.spawn`` for tests and small drivers (:func:`spawn`, picks a free port on 127.0.0.1).

On ROCm the ``"nccl"`` backend *is* RCCL (xGMI peer-to-peer between the 8 GPUs of a node).
"""

from __future__ import annotations

import datetime
import os
import random
import socket
import time
from collections.abc import Callable

import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from .affinity import pin_rank_to_gpu


def _ephemeral_low() -> int:
    try:
        with open("/proc/sys/net/ipv4/ip_local_port_range") as fh:
            return int(fh.read().split()[0])
    except (OSError, ValueError, IndexError):
        return 32768


def find_free_port() -> int:
    """A bindable TCP port on 127.0.0.1 for a rendezvous store, picked BELOW the kernel's ephemeral
    range. A port from ``bind(0)`` is ephemeral: between this probe and the store's bind (seconds of
    ``import torch`` in spawned ranks) the kernel may hand it to any outgoing connection on the box
    (RCCL bootstrap, gloo pairs, other jobs) and the store fails with EADDRINUSE -- seen once in the
    GPU suite. Ports below the range are only taken by explicit binds, so a random one that binds now
    stays free. Falls back to ``bind(0)`` if no such port binds."""
    lo = _ephemeral_low()
    rng = random.Random(os.getpid() ^ time.time_ns())
    if lo > 12000:
        for _ in range(64):
            port = rng.randrange(10000, lo)
            with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
                try:
                    s.bind(("127.0.0.1", port))
                except OSError:
                    continue
                return port
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def default_backend(device: str | torch.device | None = None) -> str:
    if device is not None:
        return "nccl" if torch.device(device).type == "cuda" else "gloo"
    return "nccl" if torch.cuda.is_available() else "gloo"


def setup_distributed(
    rank: int | None = None,
    world_size: int | None = None,
    backend: str | None = None,
    master_addr: str | None = None,
    master_port: int | str | None = None,
    timeout_s: float = 600.0,
    use_gpu: bool | None = None,
) -> tuple[int, int, torch.device]:
    """Initialise the default process group; returns ``(rank, world_size, device)``.

    Missing arguments come from the torchrun environment. Binds the process to GPU
    ``LOCAL_RANK % device_count`` before init so RCCL picks the right device.
    """
    rank = int(os.environ.get("RANK", 0)) if rank is None else rank
    world_size = int(os.environ.get("WORLD_SIZE", 1)) if world_size is None else world_size
    local_rank = int(os.environ.get("LOCAL_RANK", rank))
    os.environ["MASTER_ADDR"] = master_addr or os.environ.get("MASTER_ADDR", "127.0.0.1")
    os.environ["MASTER_PORT"] = str(master_port or os.environ.get("MASTER_PORT", "29512"))
    # async error handling: a hung/failed peer raises instead of deadlocking
    os.environ.setdefault("TORCH_NCCL_ASYNC_ERROR_HANDLING", "1")
    if backend is None:
        backend = default_backend()
    if use_gpu is None:
        use_gpu = backend == "nccl"
    if use_gpu and torch.cuda.is_available():
        # (gloo + GPU tensors: a multi-rank rehearsal with several ranks sharing one GPU)
        dev = torch.device("cuda", local_rank % torch.cuda.device_count())
        torch.cuda.set_device(dev)
    else:
        dev = torch.device("cpu")
    # host threads of this rank on the CPUs local to its GPU, before any heavy host work
    pin_rank_to_gpu(dev)
    if not dist.is_initialized():
        kw = {}
        if backend == "nccl" and dev.type == "cuda":
            kw["device_id"] = dev
        dist.init_process_group(
            backend, rank=rank, world_size=world_size, timeout=datetime.timedelta(seconds=timeout_s), **kw
        )
    return rank, world_size, dev


def cleanup_distributed() -> None:
    if dist.is_initialized():
        try:
            dist.barrier()
        finally:
            dist.destroy_process_group()


def spawn(fn: Callable, world_size: int, *args, port: int | None = None) -> None:
    """``mp.spawn`` ``fn(rank, world_size, *args)`` with a fresh 127.0.0.1 rendezvous port."""
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port or find_free_port())
    mp.spawn(fn, args=(world_size, *args), nprocs=world_size, join=True)


def supports_avg(group=None) -> bool:
    """RCCL/NCCL implement ReduceOp.AVG natively (saves the separate divide kernel); Gloo does not."""
    return dist.get_backend(group) == "nccl"


def broadcast_module_(module: torch.nn.Module, src: int = 0, group=None, buffer_mb: int = 256) -> None:
    """Broadcast every parameter of ``module`` from ``src`` with coalesced collectives (a few
    large RCCL broadcasts instead of one per tensor, reference ``:225-226``)."""
    params = [p.data for p in module.parameters()]
    if not params:
        return
    if group is None:
        group = dist.group.WORLD
    dist._broadcast_coalesced(group, params, buffer_mb * 1024 * 1024, src)


def all_reduce_mean_scalar(x: float, device) -> float:
    t = torch.tensor([x], dtype=torch.float64, device=device)
    if dist.get_backend() == "nccl":
        dist.all_reduce(t, op=dist.ReduceOp.AVG)
    else:
        dist.all_reduce(t)
        t /= dist.get_world_size()
    return float(t.item())


def all_reduce_max_scalar(x: float, device) -> float:
    t = torch.tensor([x], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())
