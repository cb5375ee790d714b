"""roctx range annotation (the reference's NVTX ranges, ``transformer_annotated.py`` and
``ddp_bucketed_overlapped_sharded.py:78-295``).

On ROCm PyTorch ``torch.cuda.nvtx`` is backed by roctx, so these ranges show up in
``rocprofv3 --marker-trace`` timelines. Annotation is off by default (zero overhead: a shared
null context) and enabled with ``CS336_ANNOTATE=1`` or :func:`enable_annotations`.
"""

from __future__ import annotations

import contextlib
import functools
import os

import torch

_ENABLED = os.environ.get("CS336_ANNOTATE", "0") == "1"
_NULL = contextlib.nullcontext()


def enable_annotations(flag: bool = True) -> None:
    global _ENABLED
    _ENABLED = flag


def annotations_enabled() -> bool:
    return _ENABLED


@contextlib.contextmanager
def _range(name: str):
    torch.cuda.nvtx.range_push(name)
    try:
        yield
    finally:
        torch.cuda.nvtx.range_pop()


def annotate(name: str):
    """``with annotate("attention"): ...`` — a roctx range when enabled, else a no-op."""
    if _ENABLED and torch.cuda.is_available():
        return _range(name)
    return _NULL


def annotated(name: str | None = None):
    """Decorator form of :func:`annotate`."""

    def deco(fn):
        label = name or fn.__qualname__

        @functools.wraps(fn)
        def wrapper(*a, **k):
            with annotate(label):
                return fn(*a, **k)

        return wrapper

    return deco
