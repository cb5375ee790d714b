"""Collective microbenchmark (reference ``distributed_communication_single.py``; handout §2.1.2).

Measures all-reduce (and optionally reduce-scatter / all-gather / broadcast) latency over sizes
1 MB … 1 GB, reporting algorithm bandwidth (bytes / time) and bus bandwidth
(algbw · 2(W-1)/W for all-reduce, (W-1)/W for RS/AG), the max over ranks of the mean time.
On MI355X the backend is RCCL over xGMI (7 point-to-point links per GPU); the CPU path (Gloo)
reproduces the reference's committed configuration (W=2, 1/10/100 MB).

    torchrun --nproc-per-node 8 --master-addr 127.0.0.1 -m cs336_systems.bench.collectives --sizes-mb 1 10 100 1024
    python -m cs336_systems.bench.collectives --cpu --world-size 2 --sizes-mb 1 10 100
"""

from __future__ import annotations

import argparse
import json
import os
import time

import torch
import torch.distributed as dist

from ..parallel.comm import cleanup_distributed, setup_distributed, spawn


def _busbw_factor(op: str, w: int) -> float:
    if op == "all_reduce":
        return 2.0 * (w - 1) / w
    if op in ("reduce_scatter", "all_gather"):
        return (w - 1) / w
    return 1.0


def run_collective(op: str, nbytes: int, dev, warmup: int, iters: int, dtype=torch.float32) -> float:
    """Mean seconds per collective on this rank."""
    w = dist.get_world_size()
    n = max(1, nbytes // torch.tensor([], dtype=dtype).element_size())
    n = (n // w) * w or w
    x = torch.rand(n, dtype=dtype, device=dev)
    out = torch.empty(n // w, dtype=dtype, device=dev) if op == "reduce_scatter" else torch.empty(n * w if op == "all_gather" else 0, dtype=dtype, device=dev)

    def once():
        if op == "all_reduce":
            dist.all_reduce(x)
        elif op == "reduce_scatter":
            dist.reduce_scatter_tensor(out, x)
        elif op == "all_gather":
            dist.all_gather_into_tensor(out, x)
        elif op == "broadcast":
            dist.broadcast(x, 0)

    sync = (lambda: torch.cuda.synchronize(dev)) if dev.type == "cuda" else (lambda: None)
    for _ in range(warmup):
        once()
    sync()
    dist.barrier()
    t0 = time.perf_counter()
    for _ in range(iters):
        once()
    sync()
    return (time.perf_counter() - t0) / iters


def _worker(rank, world, args, backend):
    rank, world, dev = setup_distributed(rank, world, backend=backend)
    rows = _bench(rank, world, dev, args)
    if rank == 0 and args.json:
        with open(args.json, "w") as f:
            json.dump(rows, f, indent=1)
    cleanup_distributed()


def _bench(rank, world, dev, args):
    rows = []
    for op in args.ops:
        for mb in args.sizes_mb:
            nbytes = int(mb * 2**20)
            t = run_collective(op, nbytes, dev, args.warmup, args.iters)
            tt = torch.tensor([t], dtype=torch.float64, device=dev)
            dist.all_reduce(tt, op=dist.ReduceOp.MAX)
            t = float(tt.item())
            algbw = nbytes / t / 1e9
            row = dict(op=op, world=world, size_mb=mb, ms=t * 1e3, algbw_GBps=algbw, busbw_GBps=algbw * _busbw_factor(op, world), backend=dist.get_backend())
            rows.append(row)
            if rank == 0:
                print(json.dumps(row), flush=True)
    return rows


def main(argv=None):
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--sizes-mb", nargs="+", type=float, default=[1, 10, 100, 1024])
    ap.add_argument("--ops", nargs="+", default=["all_reduce"], choices=["all_reduce", "reduce_scatter", "all_gather", "broadcast"])
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--cpu", action="store_true", help="Gloo on CPU tensors via mp.spawn")
    ap.add_argument("--world-size", type=int, default=2)
    ap.add_argument("--json", default=None)
    a = ap.parse_args(argv)
    if "RANK" in os.environ and "WORLD_SIZE" in os.environ:
        rank, world, dev = setup_distributed(backend="gloo" if a.cpu else None)
        rows = _bench(rank, world, dev, a)
        if rank == 0 and a.json:
            with open(a.json, "w") as f:
                json.dump(rows, f, indent=1)
        cleanup_distributed()
    else:
        spawn(_worker, a.world_size, a, "gloo" if a.cpu or not torch.cuda.is_available() else "nccl")


if __name__ == "__main__":
    main()
