"""Attention benchmark: naive (materializing) vs ``torch.compile``d naive vs HIP FlashAttention-2
(reference ``cs336_systems/benchmark_attention.py``; handout §1.2.1 / §1.3).

Protocol per the handout: batch 8, one head, d ∈ {16, 32, 64, 128}, seq ∈ {256 … 16384};
100 forward passes and 100 backward passes timed with syncs, memory in use before the backward,
OOM rows recorded instead of aborting. Unlike the reference, ``--compile`` is honoured and the
causal flag is forwarded (reference bugs 6 / H6).

    python -m cs336_systems.bench.attention --impls naive compiled flash --seqs 256 1024 4096 16384
"""

from __future__ import annotations

import argparse
import json
import math
import time

import torch

from ..ops.flash_attention import FlashAttentionHIP, FlashAttentionTorch


class Attention(torch.nn.Module):
    """Materializing scaled-dot-product attention with a causal mask (``model.py:400-432``)."""

    def forward(self, q, k, v, is_causal: bool = True):
        d = q.shape[-1]
        s = torch.matmul(q, k.transpose(-1, -2)) / math.sqrt(d)
        if is_causal:
            n = q.shape[-2]
            mask = torch.ones(n, k.shape[-2], dtype=torch.bool, device=q.device).tril()
            s = s.masked_fill(~mask, float("-inf"))
        return torch.matmul(torch.softmax(s, dim=-1), v)


def _sync(dev):
    if torch.device(dev).type == "cuda":
        torch.cuda.synchronize()


def compare_attention_methods(seq_len: int, d_model: int, impl: str = "naive", batch: int = 8, warmup: int = 10, iters: int = 100, is_causal: bool = True, dtype=torch.float32, device=None) -> dict:
    dev = device or ("cuda" if torch.cuda.is_available() else "cpu")
    row = dict(impl=impl, seq=seq_len, d=d_model, batch=batch, causal=is_causal, dtype=str(dtype).split(".")[-1])
    try:
        torch.manual_seed(0)
        q, k, v = (torch.randn(batch, seq_len, d_model, device=dev, dtype=dtype, requires_grad=True) for _ in range(3))
        if impl == "naive":
            fn = Attention()
        elif impl == "compiled":
            fn = torch.compile(Attention())
        elif impl == "flash":
            fn = (lambda a, b, c, causal: FlashAttentionHIP.apply(a, b, c, causal)) if str(dev).startswith("cuda") else (lambda a, b, c, causal: FlashAttentionTorch.apply(a, b, c, causal))
        else:
            raise ValueError(impl)
        for _ in range(warmup):
            fn(q, k, v, is_causal).sum().backward()
        _sync(dev)
        t0 = time.perf_counter()
        for _ in range(iters):
            out = fn(q, k, v, is_causal)
        _sync(dev)
        row["fwd_ms"] = (time.perf_counter() - t0) * 1e3 / iters
        if str(dev).startswith("cuda"):
            torch.cuda.reset_peak_memory_stats()
        out = fn(q, k, v, is_causal)
        _sync(dev)
        row["mem_before_bwd_mib"] = torch.cuda.memory_allocated() / 2**20 if str(dev).startswith("cuda") else None
        bwd = 0.0
        for _ in range(iters):
            out = fn(q, k, v, is_causal)
            g = torch.ones_like(out)
            _sync(dev)
            t0 = time.perf_counter()
            out.backward(g)
            _sync(dev)
            bwd += time.perf_counter() - t0
        row["bwd_ms"] = bwd * 1e3 / iters
    except torch.OutOfMemoryError:
        row["error"] = "OOM"
    if str(dev).startswith("cuda"):
        torch.cuda.empty_cache()
    return row


def benchmark_attention(seqs=(256, 1024, 4096, 8192, 16384), ds=(16, 32, 64, 128), impls=("naive", "compiled", "flash"), **kw) -> list[dict]:
    rows = []
    for impl in impls:
        for d in ds:
            for s in seqs:
                r = compare_attention_methods(s, d, impl, **kw)
                rows.append(r)
                print(json.dumps(r), flush=True)
    return rows


def main(argv=None):
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--impls", nargs="+", default=["naive", "compiled", "flash"])
    ap.add_argument("--seqs", nargs="+", type=int, default=[256, 1024, 4096, 8192, 16384])
    ap.add_argument("--ds", nargs="+", type=int, default=[16, 32, 64, 128])
    ap.add_argument("--batch", type=int, default=8)
    ap.add_argument("--iters", type=int, default=100)
    ap.add_argument("--no-causal", action="store_true")
    ap.add_argument("--dtype", default="fp32", choices=["fp32", "bf16"])
    ap.add_argument("--json", default=None)
    a = ap.parse_args(argv)
    dt = torch.float32 if a.dtype == "fp32" else torch.bfloat16
    rows = benchmark_attention(a.seqs, a.ds, a.impls, batch=a.batch, iters=a.iters, is_causal=not a.no_causal, dtype=dt)
    if a.json:
        with open(a.json, "w") as f:
            json.dump(rows, f, indent=1)


if __name__ == "__main__":
    main()
