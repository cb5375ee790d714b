"""Memory profiling helpers (reference ``benchmark.py:175-245``, handout p.7-8).

The ROCm caching allocator implements the same memory-history recorder as CUDA, so snapshots
written here open in pytorch.org/memory_viz exactly like the reference's ``memory_files/*.pickle``.
Only files written by this code are ever unpickled (by the viewer, not by us).
"""

from __future__ import annotations

import contextlib
import os

import torch


def reset_peak(device=None) -> None:
    if torch.cuda.is_available():
        torch.cuda.synchronize(device)
        torch.cuda.empty_cache()
        torch.cuda.reset_peak_memory_stats(device)


def peak_mib(device=None) -> float:
    if not torch.cuda.is_available():
        return 0.0
    return torch.cuda.max_memory_allocated(device) / 2**20


def allocated_mib(device=None) -> float:
    if not torch.cuda.is_available():
        return 0.0
    return torch.cuda.memory_allocated(device) / 2**20


@contextlib.contextmanager
def record_memory_history(path: str | None, max_entries: int = 1_000_000):
    """Record allocator history inside the block and dump a snapshot to ``path`` (if given)."""
    if path is None or not torch.cuda.is_available():
        yield
        return
    torch.cuda.memory._record_memory_history(max_entries=max_entries)
    try:
        yield
    finally:
        os.makedirs(os.path.dirname(os.path.abspath(path)), exist_ok=True)
        torch.cuda.memory._dump_snapshot(path)
        torch.cuda.memory._record_memory_history(enabled=None)
