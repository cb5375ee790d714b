"""Data loading (reference ``cs336-basics/cs336_basics/data.py:10-30``) and synthetic batches.

``get_batch`` keeps the reference contract (random windows of a 1-D token array, targets shifted
by one, int64 tensors on ``device``) but gathers all windows with one vectorized fancy-index read
of the (memory-mapped) array instead of a Python loop, and uses pinned memory + a non-blocking
H2D copy on GPU. ``synthetic_batch`` draws tokens directly on the device (no H2D traffic) for
benchmarks, which is what BASELINE.json's "synthetic" data means.
"""

from __future__ import annotations

import numpy as np
import numpy.typing as npt
import torch


def get_batch(dataset: npt.NDArray, batch_size: int, context_length: int, device: str) -> tuple[torch.Tensor, torch.Tensor]:
    starts = torch.randint(len(dataset) - context_length, (batch_size,)).numpy()
    idx = starts[:, None] + np.arange(context_length + 1)[None, :]
    window = torch.from_numpy(np.asarray(dataset[idx]).astype(np.int64))
    x, y = window[:, :-1], window[:, 1:]
    if "cuda" in str(device):
        x = x.contiguous().pin_memory().to(device, non_blocking=True)
        y = y.contiguous().pin_memory().to(device, non_blocking=True)
    else:
        x, y = x.contiguous().to(device), y.contiguous().to(device)
    return x, y


def synthetic_batch(batch_size: int, context_length: int, vocab_size: int, device, generator: torch.Generator | None = None):
    """Random token ids on ``device``: (inputs, targets) with targets = inputs shifted by one."""
    toks = torch.randint(0, vocab_size, (batch_size, context_length + 1), device=device, generator=generator)
    return toks[:, :-1].contiguous(), toks[:, 1:].contiguous()
