"""Emulated W = 8 bucketed DDP on ONE GPU: the XL training step of bench.py under DDPBucketed
(cs336_systems/parallel/ddp.py), with every bucket's all-reduce replaced by an RCCL-shaped occupant
on a communication stream -- ``channels`` workgroups of an RCCL gfx950 channel block (256 threads,
21,184 B LDS) held for the time the ring all-reduce of that bucket would take over xGMI
(``2·(W-1)/W · bytes / busbw + latency``; csrc/ops/occupy.hip). The occupant takes CUs away from
the backward GEMMs exactly as RCCL's channel blocks do, and the main stream waits for it where
``finish_gradient_synchronization`` waits for the real collective. With ``--occupant bytes`` (the
default since round 6) the occupant also MOVES the HBM bytes of the ring on this rank -- ``hbm_factor``
x 2·(W-1)/W x bucket bytes (3: per step a ring reads two chunks and writes two, counting the chunk a
peer writes into this rank's receive buffer over xGMI), read from the bucket and written to a scratch
buffer, paced over the collective's time (``torch.ops.cs336.occupy_bytes``): the reduction's traffic
competes with the backward's memory-bound kernels as it will at W = 8. ``--occupant sleep`` is the
round-5 form (CUs and LDS taken, no bytes). Not modelled: cross-rank skew, xGMI link contention.

Prints one JSON line per (bucket cap, channels, busbw, optimizer overlap) with ms/step, next to the
plain step (no DDP) and DDPBucketed over a real RCCL world-1 group (which issues no collective since
round 6: parallel/ddp.py).

    python scripts/comm_emulation.py [--batch 102] [--steps 6] [--caps 32 128 512] [--channels 16 32] [--busbw 300] [--overlap-opt off on]
"""

from __future__ import annotations

import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402


class _Handle:
    def __init__(self, ev):
        self.ev = ev

    def wait(self):
        torch.cuda.current_stream().wait_event(self.ev)


def make_emulated(base_cls, world: int, busbw_gbs: float, channels: int, lat_us: float, occupant: str = "bytes",
                  hbm_factor: float = 3.0):
    from cs336_systems import ops  # noqa: F401

    class EmulatedDDP(base_cls):
        comm_ms: list

        def _all_reduce(self, t, async_op):
            nbytes = t.numel() * t.element_size()
            bus = 2 * (world - 1) / world * nbytes
            ms = bus / (busbw_gbs * 1e9) * 1e3 + lat_us / 1e3
            self.__dict__.setdefault("comm_ms", []).append(ms)
            s = self.__dict__.setdefault("_comm_stream", torch.cuda.Stream())
            s.wait_stream(torch.cuda.current_stream())
            cnt = self.__dict__.setdefault("_cnt", torch.zeros(1, dtype=torch.int32, device=t.device))
            with torch.cuda.stream(s):
                if occupant == "bytes" and nbytes >= 16384:
                    scratch = self.__dict__.get("_scratch")
                    if scratch is None or scratch.numel() < t.numel():
                        scratch = torch.empty(t.numel(), dtype=t.dtype, device=t.device)
                        self.__dict__["_scratch"] = scratch
                    torch.ops.cs336.occupy_bytes(channels, 21184, ms, t, scratch, int(hbm_factor * bus), cnt)
                else:
                    torch.ops.cs336.occupy(channels, 21184, ms, cnt)
                ev = torch.cuda.Event()
                ev.record(s)
            return _Handle(ev)

    return EmulatedDDP


def run(args, cap, channels, busbw, mode, overlap=False):
    from cs336_systems import ops
    from cs336_systems.models import build_model
    from cs336_systems.parallel.ddp import DDPBucketed

    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    model = build_model(args.model, 512, device=dev)
    ddp = None
    if mode == "real":
        ddp = DDPBucketed(model, cap)
    elif mode == "emulated":
        ddp = make_emulated(DDPBucketed, args.world, busbw, channels, args.lat_us, args.occupant, args.hbm_factor)(model, cap)
    opt = ops.FusedAdamW(model.parameters(), lr=1e-4, betas=(0.9, 0.95), eps=1e-8, weight_decay=0.01, bf16_shadows=True)
    if overlap:  # the update of each reduced bucket on the optimizer stream, during backward
        assert opt.enable_backward_overlap(ddp=ddp)
    fwd = ddp if ddp is not None else model
    x = torch.randint(0, 10000, (args.batch, 512), device=dev)
    times = []
    for i in range(args.warmup + args.steps):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        opt.zero_grad(set_to_none=True)
        with torch.autocast("cuda", dtype=torch.bfloat16):
            loss = ops.cross_entropy(fwd(x), x)
        loss.backward()
        if ddp is not None:
            ddp.finish_gradient_synchronization()
        opt.step()
        torch.cuda.synchronize()
        if i >= args.warmup:
            times.append((time.perf_counter() - t0) * 1e3)
    comm = getattr(ddp, "comm_ms", None)
    nb = len(ddp.buckets) if ddp is not None else 0
    out = {"mode": mode, "occupant": args.occupant if mode == "emulated" else None, "overlap_opt": overlap,
           "batch": args.batch, "bucket_mb": cap if ddp is not None else None,
           "channels": channels if mode == "emulated" else None,
           "busbw_gbs": busbw if mode == "emulated" else None, "buckets": nb,
           "ms_per_step": round(sorted(times)[len(times) // 2], 2),
           "emulated_comm_ms_per_step": round(sum(comm) / (args.warmup + args.steps), 2) if comm else None}
    if ddp is not None:
        ddp.remove_hooks()
    del ddp, opt, model, loss
    import gc

    gc.collect()
    torch.cuda.empty_cache()
    return out


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="xl")
    ap.add_argument("--batch", type=int, default=102)
    ap.add_argument("--steps", type=int, default=6)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--world", type=int, default=8)
    ap.add_argument("--caps", type=float, nargs="+", default=[32, 128, 512])
    ap.add_argument("--channels", type=int, nargs="+", default=[16, 32])
    ap.add_argument("--busbw", type=float, nargs="+", default=[300.0])
    ap.add_argument("--lat-us", type=float, default=25.0)
    ap.add_argument("--occupant", choices=["bytes", "sleep"], default="bytes")
    ap.add_argument("--hbm-factor", type=float, default=3.0, help="HBM bytes per bus byte of the ring, this rank")
    ap.add_argument("--overlap-opt", nargs="+", default=["off", "on"], choices=["off", "on"])
    a = ap.parse_args()
    from cs336_systems import ops

    assert ops.load_ext(), ops.load_error()
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29613")
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
    print(json.dumps(run(a, None, 0, 0, "none")), flush=True)
    for ov in a.overlap_opt:
        print(json.dumps(run(a, 128.0, 0, 0, "real", ov == "on")), flush=True)
    for bw in a.busbw:
        for ch in a.channels:
            for cap in a.caps:
                for ov in a.overlap_opt:
                    print(json.dumps(run(a, cap, ch, bw, "emulated", ov == "on")), flush=True)
    dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
