"""Training checkpoints: model + optimizer (+ ZeRO-1 shards) + step, with atomic resume.

The reference has no resume path: it only writes ad-hoc ``*.pt`` artefacts
(``naive_ddp.py:27-33, 155-162``) and a ``from_pretrained`` model format (``model.py:312-327``).
This module adds what a multi-GPU training job needs:

* ``<dir>/step_<n>/model.pt`` — the (replicated) model state dict, written by rank 0;
* ``<dir>/step_<n>/optim.pt`` — the optimizer state, rank 0 (replicated optimizers), or
  ``optim_rank<r>.pt`` per rank for :class:`~cs336_systems.parallel.ShardedOptimizer` (each rank
  owns a disjoint shard, so every rank writes its own file and nothing is gathered);
* ``<dir>/step_<n>/meta.json`` — step, world size, sharding flag and user metadata;
* ``<dir>/latest`` — the name of the last COMPLETE checkpoint, replaced atomically only after
  every rank has finished writing (barrier), so a job killed mid-save resumes from the previous one.

Everything is loaded with ``torch.load(weights_only=True)``: checkpoints hold tensors and plain
containers only.
"""

from __future__ import annotations

import json
import os
import shutil

import torch
import torch.distributed as dist
import torch.nn as nn

from .parallel.sharded_optimizer import ShardedOptimizer


def _rank_world() -> tuple[int, int]:
    if dist.is_available() and dist.is_initialized():
        return dist.get_rank(), dist.get_world_size()
    return 0, 1


def _barrier() -> None:
    if dist.is_available() and dist.is_initialized():
        dist.barrier()


def _unwrap(model: nn.Module) -> nn.Module:
    m = getattr(model, "module", model)
    return getattr(m, "_orig_mod", m)


def _atomic_save(obj, path: str) -> None:
    tmp = path + ".tmp"
    torch.save(obj, tmp)
    os.replace(tmp, path)


def save_checkpoint(ckpt_dir: str, step: int, model: nn.Module, optimizer: torch.optim.Optimizer | None = None, meta: dict | None = None, keep: int = 2,
                    model_state: dict | None = None, sharded: bool | None = None) -> str:
    """Collective: every rank must call it. Returns the checkpoint directory. ``model_state``
    overrides ``model.state_dict()`` (e.g. the gathered state of a tensor-parallel model) and
    ``sharded=True`` writes one optimizer file per rank whatever the optimizer type."""
    rank, world = _rank_world()
    name = f"step_{step:08d}"
    path = os.path.join(ckpt_dir, name)
    if rank == 0:
        os.makedirs(path, exist_ok=True)
    _barrier()
    sharded = (_is_sharded(optimizer) if sharded is None else sharded) and world > 1
    if rank == 0:
        _atomic_save(model_state if model_state is not None else _unwrap(model).state_dict(), os.path.join(path, "model.pt"))
    if optimizer is not None:
        if sharded:
            _atomic_save(optimizer.state_dict(), os.path.join(path, f"optim_rank{rank}.pt"))
        elif rank == 0:
            _atomic_save(optimizer.state_dict(), os.path.join(path, "optim.pt"))
    _barrier()
    if rank == 0:
        info = dict(step=step, world_size=world, sharded_optimizer=sharded, **(meta or {}))
        with open(os.path.join(path, "meta.json"), "w") as f:
            json.dump(info, f, indent=1)
        tmp = os.path.join(ckpt_dir, "latest.tmp")
        with open(tmp, "w") as f:
            f.write(name)
        os.replace(tmp, os.path.join(ckpt_dir, "latest"))
        if keep > 0:
            old = sorted(d for d in os.listdir(ckpt_dir) if d.startswith("step_") and d != name)
            for d in old[: max(0, len(old) - (keep - 1))]:
                shutil.rmtree(os.path.join(ckpt_dir, d), ignore_errors=True)
    _barrier()
    return path


def _is_sharded(optimizer) -> bool:
    """Per-rank optimizer state: ZeRO-1 (ShardedOptimizer) or ZeRO-2 (``ZeroDDP.optimizer``)."""
    return isinstance(optimizer, ShardedOptimizer) or getattr(optimizer, "sharded_state", False)


def latest_checkpoint(ckpt_dir: str) -> str | None:
    p = os.path.join(ckpt_dir, "latest")
    if not os.path.exists(p):
        return None
    with open(p) as f:
        name = f.read().strip()
    path = os.path.join(ckpt_dir, name)
    return path if os.path.exists(os.path.join(path, "meta.json")) else None


def load_checkpoint(path: str, model: nn.Module, optimizer: torch.optim.Optimizer | None = None, map_location="cpu") -> dict:
    """Load into ``model`` (and ``optimizer``); returns ``meta`` (``meta['step']`` = the step the
    checkpoint was taken after). A sharded checkpoint must be loaded at the same world size."""
    with open(os.path.join(path, "meta.json")) as f:
        meta = json.load(f)
    sd = torch.load(os.path.join(path, "model.pt"), map_location=map_location, weights_only=True)
    _unwrap(model).load_state_dict(sd)
    if optimizer is not None:
        load_optimizer_state(path, optimizer, map_location, meta)
    return meta


def load_optimizer_state(path: str, optimizer: torch.optim.Optimizer, map_location="cpu", meta: dict | None = None) -> None:
    """The optimizer half of :func:`load_checkpoint` (ZeRO-2 builds its optimizer only after the
    model weights are loaded and re-homed into its buckets)."""
    rank, world = _rank_world()
    if meta is None:
        with open(os.path.join(path, "meta.json")) as f:
            meta = json.load(f)
    if meta["sharded_optimizer"]:
        if meta["world_size"] != world:
            raise ValueError(f"sharded optimizer checkpoint was written by {meta['world_size']} ranks, loading on {world}")
        osd = torch.load(os.path.join(path, f"optim_rank{rank}.pt"), map_location=map_location, weights_only=True)
    else:
        osd = torch.load(os.path.join(path, "optim.pt"), map_location=map_location, weights_only=True)
    optimizer.load_state_dict(osd)
    _state_to_param_device(optimizer)


def _state_to_param_device(optimizer: torch.optim.Optimizer) -> None:
    """``Optimizer.load_state_dict`` casts floating state to the param dtype/device already; this
    also moves any leftover tensors of the wrapped local optimizer of a ShardedOptimizer."""
    inner = optimizer.optimizer if isinstance(optimizer, ShardedOptimizer) else optimizer
    if inner is None:
        return
    for p, st in inner.state.items():
        for k, v in st.items():
            if torch.is_tensor(v) and v.device != p.device and v.dim() > 0:
                st[k] = v.to(p.device)
