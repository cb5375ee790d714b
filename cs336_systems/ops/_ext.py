"""Loader for the in-tree HIP extension (``cs336_systems/_native/libcs336_hip.so``).

The extension registers its kernels as ``torch.ops.cs336.*`` through ``TORCH_LIBRARY`` (see
``csrc/bindings.cpp``); it is built by ``cs336_systems/_native/build.py`` with hipcc for gfx950.

Backend policy (``CS336_BACKEND`` env var or :func:`set_backend`):

* ``"auto"`` (default): GPU tensors use the HIP kernels; CPU tensors use the eager PyTorch
  reference implementations. If a GPU tensor reaches an op and the extension cannot be loaded,
  the op raises (no silent fallback on a GPU box).
* ``"torch"``: force the eager PyTorch implementations everywhere (A/B benchmarking only).
* ``"hip"``: like auto, but also raise if the extension is missing on a CPU-only box when an op
  is called with a CUDA tensor.
"""

from __future__ import annotations

import os
import threading
from contextlib import contextmanager

import torch

_LIB_NAME = "libcs336_hip.so"
_LIB_DIR = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "_native")
# CS336_LIB: load a variant build instead (A/B runs, cs336_systems/_native/build.py CS336_BUILD_VARIANT)
LIB_PATH = os.environ.get("CS336_LIB") or os.path.join(_LIB_DIR, _LIB_NAME)

_lock = threading.Lock()
_loaded: bool | None = None
_load_error: str | None = None
_backend = os.environ.get("CS336_BACKEND", "auto").lower()


def load_ext() -> bool:
    """Load the HIP extension once; returns True if ``torch.ops.cs336`` is available."""
    global _loaded, _load_error
    if _loaded is not None:
        return _loaded
    with _lock:
        if _loaded is not None:
            return _loaded
        if not os.path.exists(LIB_PATH):
            _loaded, _load_error = False, f"{LIB_PATH} not built (run `python -m cs336_systems._native.build`)"
            return False
        try:
            torch.ops.load_library(LIB_PATH)
            from . import _fake  # noqa: F401  (registers fake/meta impls for torch.compile)

            _loaded = True
            # explicit Inductor fallbacks for the HIP ops (models/compiled.py explains why); an
            # optimization of compile time only, so it can never fail the load
            try:
                from ..models.compiled import register_inductor_fallbacks

                register_inductor_fallbacks(("cs336",))
            except Exception:  # noqa: BLE001
                pass
        except Exception as e:  # pragma: no cover - depends on the box
            _loaded, _load_error = False, f"failed to load {LIB_PATH}: {e!r}"
    return _loaded


def ext_available() -> bool:
    return load_ext()


def load_error() -> str | None:
    load_ext()
    return _load_error


def get_backend() -> str:
    return _backend


def set_backend(name: str) -> None:
    global _backend
    name = name.lower()
    if name not in ("auto", "torch", "hip"):
        raise ValueError(f"unknown backend {name!r}")
    _backend = name


@contextmanager
def backend(name: str):
    prev = get_backend()
    set_backend(name)
    try:
        yield
    finally:
        set_backend(prev)


def use_hip(*tensors: torch.Tensor) -> bool:
    """Decide whether an op on ``tensors`` runs the HIP kernel.

    GPU tensors always go to HIP unless the backend is forced to ``torch``; a missing extension
    on a GPU tensor is an error, never a silent fallback.
    """
    if _backend == "torch":
        return False
    on_gpu = any(t is not None and t.is_cuda for t in tensors)
    if not on_gpu:
        return False
    if not load_ext():
        raise RuntimeError(
            "cs336 HIP extension is required for GPU tensors but is unavailable: " f"{_load_error}"
        )
    return True


def ops():
    """``torch.ops.cs336`` namespace (loads the extension)."""
    if not load_ext():
        raise RuntimeError(f"cs336 HIP extension unavailable: {_load_error}")
    return torch.ops.cs336
