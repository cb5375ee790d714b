"""Timing utilities: HIP-event ``do_bench`` (the reference used ``triton.testing.do_bench``,
``flashattentioncode.py:49-64``; handout leaderboard protocol p.22) and a wall-clock step timer.

``do_bench`` flushes the 256 MiB Infinity Cache + L2 between repetitions by writing a 512 MiB
scratch buffer, so kernels are timed from cold caches like Triton's harness does, and returns
per-repetition times in milliseconds measured by HIP events.
"""

from __future__ import annotations

import statistics
import time
from collections.abc import Callable
from dataclasses import dataclass, field

import torch

_FLUSH = {}


def _flush_buffer(device) -> torch.Tensor:
    key = str(device)
    if key not in _FLUSH:
        _FLUSH[key] = torch.empty(512 * 1024 * 1024 // 4, dtype=torch.int32, device=device)
    return _FLUSH[key]


def sync(device=None) -> None:
    if torch.cuda.is_available() and (device is None or torch.device(device).type == "cuda"):
        torch.cuda.synchronize(device)


def do_bench(
    fn: Callable[[], object],
    warmup: int = 25,
    rep: int = 100,
    flush_cache: bool = True,
    quantiles=(0.5, 0.2, 0.8),
    return_all: bool = False,
):
    """Time ``fn`` on the current HIP stream. Returns the median (and quantiles) in ms."""
    if not torch.cuda.is_available():
        return _cpu_bench(fn, warmup, rep, quantiles, return_all)
    dev = torch.cuda.current_device()
    buf = _flush_buffer(dev) if flush_cache else None
    for _ in range(warmup):
        fn()
    torch.cuda.synchronize()
    starts = [torch.cuda.Event(enable_timing=True) for _ in range(rep)]
    ends = [torch.cuda.Event(enable_timing=True) for _ in range(rep)]
    for i in range(rep):
        if buf is not None:
            buf.zero_()
        starts[i].record()
        fn()
        ends[i].record()
    torch.cuda.synchronize()
    times = [s.elapsed_time(e) for s, e in zip(starts, ends)]
    return _summarize(times, quantiles, return_all)


def _cpu_bench(fn, warmup, rep, quantiles, return_all):
    for _ in range(warmup):
        fn()
    times = []
    for _ in range(rep):
        t0 = time.perf_counter()
        fn()
        times.append((time.perf_counter() - t0) * 1e3)
    return _summarize(times, quantiles, return_all)


def _summarize(times, quantiles, return_all):
    if return_all:
        return times
    ts = sorted(times)
    q = [ts[min(len(ts) - 1, int(round(x * (len(ts) - 1))))] for x in quantiles]
    return q[0] if len(q) == 1 else tuple(q)


@dataclass
class StepTimer:
    """Accumulates wall-clock durations (ms) of named phases with device syncs at boundaries,
    matching the reference's ``timeit.default_timer`` + ``torch.cuda.synchronize`` protocol
    (``benchmark.py:91-117``)."""

    device: object = None
    records: dict[str, list[float]] = field(default_factory=dict)

    def time(self, name: str):
        timer = self

        class _Ctx:
            def __enter__(self_inner):
                sync(timer.device)
                self_inner.t0 = time.perf_counter()

            def __exit__(self_inner, *exc):
                sync(timer.device)
                timer.records.setdefault(name, []).append((time.perf_counter() - self_inner.t0) * 1e3)

        return _Ctx()

    def summary(self) -> dict[str, tuple[float, float]]:
        out = {}
        for k, v in self.records.items():
            out[k] = (statistics.fmean(v), statistics.pstdev(v) if len(v) > 1 else 0.0)
        return out
