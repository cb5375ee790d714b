"""Data-parallel training driver (reference ``naive_ddp.py`` train/train_ddp/train_ddp_flat and
``ddp_bucketed_overlapped_sharded.py`` train_process/train_process_ddp; handout §2.2-2.3).

Trains the Transformer LM with one of the DP variants and reports per-step time split into
forward / backward / gradient-communication wait / optimizer, the communication fraction, loss,
and peak memory after init / before the optimizer step / after it (the sharded-optimizer
accounting of handout §2.3.1). Ranks come from torchrun's env or ``--world-size`` (mp.spawn);
``--cpu`` runs Gloo on CPU (the reference's tested configuration), otherwise RCCL on GPU.

Correctness mode (``--check``): every rank also trains an unwrapped replica on the full global
batch and asserts the DP model's parameters match it after every step (what the reference's
``naive_ddp.main`` meant to do before its NameError).

    torchrun --nproc-per-node 8 --master-addr 127.0.0.1 -m cs336_systems.bench.ddp --variant bucketed --size xl --ctx 512 --batch 128
    python -m cs336_systems.bench.ddp --cpu --world-size 2 --size tiny --ctx 32 --batch 8 --variant naive --check
"""

from __future__ import annotations

import argparse
import copy
import contextlib
import gc
import json
import os
import statistics
import time

import torch
import torch.distributed as dist

from .. import ops
from ..data import synthetic_batch
from ..models import build_model
from ..parallel import DDP_VARIANTS, DEFAULT_BUCKET_MB, ShardedOptimizer, cleanup_distributed, setup_distributed, spawn, wrap_ddp
from ..utils.profiling import annotate


def _sync(dev):
    if dev.type == "cuda":
        torch.cuda.synchronize(dev)


def _mem(dev):
    return torch.cuda.memory_allocated(dev) / 2**20 if dev.type == "cuda" else 0.0


def _peak(dev):
    return torch.cuda.max_memory_allocated(dev) / 2**20 if dev.type == "cuda" else 0.0


def train_ddp(rank: int, world: int, args) -> dict | None:
    backend = "gloo" if (args.cpu or args.gloo_gpu) else None
    rank, world, dev = setup_distributed(rank, world, backend=backend, use_gpu=True if args.gloo_gpu else None)
    torch.manual_seed(args.seed)
    model = build_model(args.size, args.ctx, device=dev)
    if args.check:
        ref = copy.deepcopy(model)
        for p in ref.parameters():
            dist.broadcast(p.data, 0)
        # Adam normalizes each update to ~lr, so summation-order differences in near-zero gradient
        # entries can move a parameter by up to ~2*lr per step: scale the tolerance accordingly
        check_tol = args.check_tol if args.check_tol is not None else 2.0 * args.lr * (args.steps + args.warmup) + 1e-6
    ddp = wrap_ddp(model, args.variant, bucket_size_mb=args.bucket_mb)
    okw = dict(lr=args.lr, betas=(0.9, 0.95), eps=1e-8, weight_decay=args.wd)
    # bf16 weight shadows (models/fused.py) whenever the step runs under bf16 autocast on GPU
    shadows = (not args.cpu) and args.dtype == "bf16" and dev.type == "cuda"
    if args.sharded:
        opt = ShardedOptimizer(model.parameters(), ops.FusedAdamW, bf16_shadows=shadows, **okw).attach(ddp)
    else:
        opt = ops.FusedAdamW(model.parameters(), bf16_shadows=shadows, **okw)
        if args.overlap_opt and args.clip == 0:
            # AdamW per reduced bucket during backward (needs an AVG backend: RCCL)
            opt.enable_backward_overlap(ddp=ddp if args.variant == "bucketed" else None)
    ref_opt = ops.FusedAdamW(ref.parameters(), **okw) if args.check else None
    mem_init = _mem(dev)
    assert args.batch % world == 0, "global batch must divide by world size"
    local = args.batch // world
    gen = torch.Generator(device=dev)
    gen.manual_seed(args.seed)  # same global batches on every rank; each rank slices its part
    amp = (not args.cpu) and args.dtype == "bf16"
    autocast = (lambda: torch.autocast(dev.type, dtype=torch.bfloat16)) if amp else contextlib.nullcontext
    rec = {k: [] for k in ("fwd", "bwd", "comm", "opt", "step")}
    losses, mem_before, mem_after = [], [], []
    for it in range(args.warmup + args.steps):
        x, y = synthetic_batch(args.batch, args.ctx, 10000, dev, gen)
        xs, ys = x[rank * local : (rank + 1) * local], y[rank * local : (rank + 1) * local]
        timed = it >= args.warmup
        _sync(dev)
        t0 = time.perf_counter()
        if hasattr(ddp, "zero_grad") and args.variant in ("bucketed", "flat"):
            ddp.zero_grad()
        else:
            opt.zero_grad(set_to_none=True)
        with autocast():
            loss = ops.cross_entropy(ddp(xs), ys)
        _sync(dev)
        t1 = time.perf_counter()
        with annotate("backward"):
            loss.backward()
        _sync(dev)
        t2 = time.perf_counter()
        with annotate("grad_sync"):
            ddp.finish_gradient_synchronization()
        _sync(dev)
        t3 = time.perf_counter()
        if args.clip > 0:
            ops.clip_grad_norm_(model.parameters(), args.clip)
        mem_before.append(_peak(dev))
        opt.step()
        _sync(dev)
        t4 = time.perf_counter()
        mem_after.append(_peak(dev))
        if timed:
            for k, v in zip(("fwd", "bwd", "comm", "opt", "step"), (t1 - t0, t2 - t1, t3 - t2, t4 - t3, t4 - t0)):
                rec[k].append(v * 1e3)
        lt = loss.detach().clone()
        if dist.get_backend() == "nccl":
            dist.all_reduce(lt, op=dist.ReduceOp.AVG)
        else:
            dist.all_reduce(lt)
            lt /= world
        losses.append(float(lt))
        if args.check:
            ref_opt.zero_grad(set_to_none=True)
            with autocast():
                ops.cross_entropy(ref(x), y).backward()
            if args.clip > 0:
                ops.clip_grad_norm_(ref.parameters(), args.clip)
            ref_opt.step()
            worst = max((a - b).abs().max().item() for a, b in zip(model.parameters(), ref.parameters()))
            assert worst < check_tol, f"rank {rank} step {it}: DP params diverge from single-process ({worst:.3e})"
    out = None
    stats = {k: (statistics.fmean(v) if v else 0.0) for k, v in rec.items()}
    t = torch.tensor([stats[k] for k in ("fwd", "bwd", "comm", "opt", "step")], dtype=torch.float64, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    if rank == 0:
        fwd, bwd, comm, optt, step = (float(v) for v in t.tolist())
        out = dict(
            variant=args.variant,
            sharded=args.sharded,
            world=world,
            size=args.size,
            ctx=args.ctx,
            global_batch=args.batch,
            bucket_mb=args.bucket_mb if args.variant == "bucketed" else None,
            fwd_ms=fwd,
            bwd_ms=bwd,
            comm_wait_ms=comm,
            opt_ms=optt,
            step_ms=step,
            comm_fraction=comm / step if step else 0.0,
            tokens_per_s=args.batch * args.ctx / (step / 1e3) if step else 0.0,
            final_loss=losses[-1],
            mem_after_init_mib=mem_init,
            peak_before_step_mib=max(mem_before) if mem_before else 0.0,
            peak_after_step_mib=max(mem_after) if mem_after else 0.0,
            checked=bool(args.check),
        )
        print(json.dumps(out), flush=True)
        if args.json:
            with open(args.json, "w") as f:
                json.dump(out, f, indent=1)
    cleanup_distributed()
    return out


SWEEP_VARIANTS = (("naive", None), ("flat", None), ("individual", None), ("bucketed", 1.0), ("bucketed", 10.0),
                  ("bucketed", 100.0), ("bucketed", 1000.0))


def sweep_variants(model_name: str, ctx: int, per_rank_batch: int, dev: torch.device, *, steps: int = 2,
                   warmup: int = 1, amp: bool = True, vocab: int = 10000, budget_s: float = 60.0,
                   variants=SWEEP_VARIANTS, zero1: bool = True) -> dict:
    """The handout's multi-GPU DDP comparison on an already-initialised process group (reference
    ``naive_ddp.py:269-442, 444-634``; ``ddp_bucketed_overlapped_sharded.py:131-214, 366-419``;
    handout p.27-31, p.34-35): per variant (naive, flat, per-parameter, bucketed at each bucket
    size) ``warmup`` + ``steps`` full steps of a fresh model at ``per_rank_batch`` sequences per rank,
    reporting ms/step and the exposed gradient-communication wait (max over ranks); then ZeRO-1
    (:class:`ShardedOptimizer` over bucketed DDP) memory after init / peak before / after the
    optimizer step. Stops issuing new variants once ``budget_s`` of wall time is spent (the rest are
    reported as skipped); every rank takes the same decisions (rank 0's clock is broadcast)."""
    t_start = time.perf_counter()
    world, rank = dist.get_world_size(), dist.get_rank()
    rows, mem = [], None
    gen = torch.Generator(device=dev)
    gen.manual_seed(4321 + rank)
    autocast = (lambda: torch.autocast(dev.type, dtype=torch.bfloat16)) if amp else contextlib.nullcontext

    def over_budget() -> bool:
        t = torch.tensor([time.perf_counter() - t_start], dtype=torch.float64,
                         device=dev if dist.get_backend() == "nccl" else "cpu")
        dist.broadcast(t, 0)
        return float(t.item()) > budget_s

    def run(variant, bucket_mb, sharded=False):
        torch.manual_seed(1234)
        model = build_model(model_name, ctx, vocab_size=vocab, device=dev)
        shadows = amp and dev.type == "cuda"
        if dev.type == "cuda":
            torch.cuda.reset_peak_memory_stats(dev)
        ddp = wrap_ddp(model, variant, bucket_size_mb=bucket_mb)
        okw = dict(lr=1e-4, betas=(0.9, 0.95), eps=1e-8, weight_decay=0.01)
        if sharded:
            opt = ShardedOptimizer(model.parameters(), ops.FusedAdamW, bf16_shadows=shadows, **okw).attach(ddp)
        else:
            opt = ops.FusedAdamW(model.parameters(), bf16_shadows=shadows, **okw)
        _sync(dev)
        mem_init = _mem(dev)
        x, y = synthetic_batch(per_rank_batch, ctx, vocab, dev, gen)
        step_ms, comm_ms, before, after = [], [], [], []
        for it in range(warmup + steps):
            _sync(dev)
            t0 = time.perf_counter()
            opt.zero_grad(set_to_none=True)
            with autocast():
                loss = ops.cross_entropy(ddp(x), y)
            loss.backward()
            _sync(dev)
            t1 = time.perf_counter()
            ddp.finish_gradient_synchronization()
            _sync(dev)
            t2 = time.perf_counter()
            before.append(_peak(dev))
            opt.step()
            _sync(dev)
            t3 = time.perf_counter()
            after.append(_peak(dev))
            if it >= warmup:
                step_ms.append((t3 - t0) * 1e3)
                comm_ms.append((t2 - t1) * 1e3)
        t = torch.tensor([statistics.fmean(step_ms), statistics.fmean(comm_ms), mem_init, max(before), max(after)],
                         dtype=torch.float64, device=dev if dist.get_backend() == "nccl" else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        # the DDP hooks live in the parameters and hold the wrapper and so the model: without
        # removing them every variant's 2 B-parameter model stayed allocated (XL world-1 sweep: 138
        # GiB allocated after the ZeRO-1 model's init, profiles/r5_ddp_sweep_xl_world1.md)
        ddp.remove_hooks()
        del ddp, opt, model, loss
        gc.collect()
        if dev.type == "cuda":
            torch.cuda.empty_cache()
        return [float(v) for v in t.tolist()]

    def note(msg):
        if rank == 0:
            print(f"ddp sweep: {msg} ({time.perf_counter() - t_start:.1f} s)", file=__import__("sys").stderr, flush=True)

    def failed_anywhere(local_error: bool) -> bool:
        """Every rank learns whether any rank's variant raised. A rank that raised (an OOM inside
        run(), say) left its peers inside collectives of that variant; continuing on the failing rank
        alone would pair its next collectives with theirs. So after a failure anywhere the
        whole sweep stops, together, on every rank."""
        f = torch.tensor([1.0 if local_error else 0.0], dtype=torch.float64,
                         device=dev if dist.get_backend() == "nccl" else "cpu")
        dist.all_reduce(f, op=dist.ReduceOp.MAX)
        return f.item() > 0

    aborted = False
    for variant, bucket_mb in variants:
        row = {"variant": variant, "bucket_mb": bucket_mb}
        note(f"{variant} {bucket_mb if bucket_mb is not None else ''}")
        if aborted:
            row["skipped"] = "an earlier variant failed on some rank"
        elif over_budget():
            row["skipped"] = "time budget"
        else:
            err = None
            t_var = time.perf_counter()
            try:
                st, cw, *_ = run(variant, bucket_mb)
                row.update(ms_per_step=round(st, 3), comm_wait_ms=round(cw, 3),
                           comm_fraction=round(cw / st, 4) if st else 0.0,
                           wall_s=round(time.perf_counter() - t_var, 2))
            except Exception as e:  # noqa: BLE001 - reported in the JSON, never loses the headline
                err = row["error"] = f"{type(e).__name__}: {e}"[:300]
            # every rank exchanges the flag, the failing one included: an error raised at a variant
            # boundary (model build, OOM before the first bucket) stops the sweep on all ranks
            # together; one raised inside a collective sequence leaves the peers in that sequence,
            # where bench.py's SweepWatchdog bounds the wait and marks the sweep timed out
            if failed_anywhere(err is not None):
                aborted = True
                row.setdefault("error", "failed on another rank")
        rows.append(row)
    if aborted:
        zero1 = False
        mem = {"skipped": "an earlier variant failed on some rank"}
    if zero1:
        if over_budget():
            mem = {"skipped": "time budget"}
        else:
            try:
                t_var = time.perf_counter()
                _, _, m0, mb, ma = run("bucketed", DEFAULT_BUCKET_MB, sharded=True)
                _, _, r0, rb, ra = run("bucketed", DEFAULT_BUCKET_MB, sharded=False)
                zero1_wall = round(time.perf_counter() - t_var, 2)
                mem = {"zero1": {"after_init_mib": round(m0, 1), "peak_before_step_mib": round(mb, 1),
                                 "peak_after_step_mib": round(ma, 1)},
                       "replicated": {"after_init_mib": round(r0, 1), "peak_before_step_mib": round(rb, 1),
                                      "peak_after_step_mib": round(ra, 1)},
                       "bucket_mb": DEFAULT_BUCKET_MB, "wall_s": zero1_wall}
            except Exception as e:  # noqa: BLE001
                mem = {"error": f"{type(e).__name__}: {e}"[:300]}
    return {"model": model_name, "ctx": ctx, "per_rank_batch": per_rank_batch, "steps": steps, "warmup": warmup,
            "world": world, "variants": rows, "zero1_memory": mem,
            "wall_s": round(time.perf_counter() - t_start, 2)}


def _spawned(rank, world, args):
    train_ddp(rank, world, args)


def parse(argv=None):
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--variant", default="bucketed", choices=sorted(DDP_VARIANTS))
    ap.add_argument("--bucket-mb", type=float, default=DEFAULT_BUCKET_MB)
    ap.add_argument("--sharded", action="store_true")
    ap.add_argument("--overlap-opt", action="store_true", help="AdamW overlapped with backward (bucketed: per reduced bucket)")
    ap.add_argument("--size", default="xl")
    ap.add_argument("--ctx", type=int, default=512)
    ap.add_argument("--batch", type=int, default=16, help="global batch (split over ranks)")
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--lr", type=float, default=1e-4)
    ap.add_argument("--wd", type=float, default=0.01)
    ap.add_argument("--clip", type=float, default=0.0)
    ap.add_argument("--dtype", default="bf16", choices=["bf16", "fp32"])
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--cpu", action="store_true")
    ap.add_argument("--gloo-gpu", action="store_true", help="gloo over GPU tensors: several ranks may share one GPU")
    ap.add_argument("--world-size", type=int, default=2)
    ap.add_argument("--check", action="store_true")
    ap.add_argument("--check-tol", type=float, default=None)
    ap.add_argument("--json", default=None)
    return ap.parse_args(argv)


def main(argv=None):
    args = parse(argv)
    if "RANK" in os.environ and "WORLD_SIZE" in os.environ:
        train_ddp(int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"]), args)
    else:
        spawn(_spawned, args.world_size, args)


if __name__ == "__main__":
    main()
