"""Data-parallel Transformer-LM training driver with checkpoint/resume.

The reference trains through ad-hoc scripts with hard-coded hparams
(``ddp_bucketed_overlapped_sharded.py:367-404``, ``naive_ddp.py:662-684``) and cannot resume.
This driver is one torchrun-compatible entry point over the framework's pieces:

* model: :func:`cs336_systems.models.build_model` (registry size or explicit dims), bf16 autocast
  over fp32 master weights, HIP kernels on GPU;
* data parallelism: any of the four DP variants (``--ddp``) and optional ZeRO-1 (``--sharded``),
  or ZeRO-2 (``--ddp zero``: reduce-scattered gradients, sharded fused AdamW, parameter
  all-gather under the next forward; ``parallel/zero.py``);
* tensor parallelism (``--tensor-parallel``): heads and d_ff sharded over all ranks
  (``parallel/tensor_parallel.py``), every rank on the whole batch, checkpoints hold the gathered
  weights and one optimizer shard per rank;
* context parallelism (``--context-parallel``, ``--cp-layout zigzag|contiguous``): each sequence is
  split over the ranks and attention runs as ring attention (``parallel/context_parallel.py``);
  the DP wrapper still averages the (replicated) weights' gradients;
* HIP graphs (``--graphs``, single process on GPU): forward + loss + backward replayed from one
  captured graph (``utils/graphs.py``), the optimizer stepping eagerly after each replay;
* optimizer: fused HIP AdamW (bf16 weight shadows on GPU), cosine LR with warmup, global-norm
  clipping;
* data: a 1-D token file (``.npy`` or raw ``uint16`` ``.bin``, memory-mapped) or synthetic tokens;
  batch ``s`` is drawn from a generator seeded by ``(seed, s)``, identical on every rank (each rank
  takes its slice), so a resumed run replays exactly the batches the uninterrupted run would have;
* checkpoints: :mod:`cs336_systems.checkpoint` every ``--ckpt-every`` steps and at the end;
  ``--resume`` continues from ``<ckpt-dir>/latest``;
* failure handling: process-group timeout + async error handling (``setup_distributed``), a
  non-finite loss aborts the job (no checkpoint is written over a good one).

Usage::

    torchrun --nproc-per-node 8 --master-addr 127.0.0.1 -m cs336_systems.train --size xl --ctx 512 \
        --batch 192 --steps 1000 --ddp bucketed --ckpt-dir ckpt/ --resume
"""

from __future__ import annotations

import argparse
import contextlib
import dataclasses
import json
import math
import os
import sys
import time

from .rccl_env import apply_multi_gpu_env

# multi-rank environment (the hipBLASLt stream-K grid cap, kept for hipBLASLt builds that honour it:
# profiles/r4_streamk_cap.md measured it inert on this image), set before torch loads hipBLASLt,
# exactly as bench.py does
_CORES_ENV = apply_multi_gpu_env(int(os.environ.get("WORLD_SIZE", "1")))

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

from . import ops  # noqa: E402
from .checkpoint import latest_checkpoint, load_checkpoint, load_optimizer_state, save_checkpoint
from .models import build_model
from .models.fused import refresh_bf16_shadows
from .parallel.tensor_parallel import tp_clip_grad_norm_
from .parallel import (
    DEFAULT_BUCKET_MB,
    ShardedOptimizer,
    ZeroDDP,
    gather_tp_state_dict,
    tensor_parallel_,
    cleanup_distributed,
    enable_context_parallel,
    setup_distributed,
    shard_sequence,
    wrap_ddp,
)


@dataclasses.dataclass
class TrainConfig:
    size: str = "small"
    ctx: int = 256
    vocab: int = 10000
    batch: int = 8  # global batch (sequences), split over ranks
    steps: int = 100
    lr: float = 3e-4
    min_lr: float = 3e-5
    warmup: int = 10
    wd: float = 0.1
    beta1: float = 0.9
    beta2: float = 0.95
    eps: float = 1e-8
    clip: float = 1.0
    dtype: str = "bf16"  # autocast dtype on GPU; "fp32" disables autocast
    ddp: str = "bucketed"
    bucket_mb: float = DEFAULT_BUCKET_MB
    sharded: bool = False
    context_parallel: bool = False  # split every sequence over the ranks (ring attention) instead of the batch
    cp_layout: str = "zigzag"
    tensor_parallel: bool = False  # shard heads / d_ff over all ranks (Megatron-style TP) instead of the batch
    graphs: bool = False  # single process on GPU: replay fwd + loss + bwd from one captured HIP graph
    data: str | None = None  # token file; None = synthetic
    seed: int = 0
    ckpt_dir: str | None = None
    ckpt_every: int = 0
    resume: bool = False
    stop_after: int = 0  # run at most this many steps in this invocation, checkpoint, exit (0 = all)
    log_every: int = 10
    log_file: str | None = None
    device: str = "auto"  # auto | cuda | cpu


def lr_at(step: int, cfg: TrainConfig) -> float:
    """Linear warmup then cosine decay to ``min_lr`` at ``steps`` (``cs336_basics.get_cosine_lr``)."""
    if step < cfg.warmup:
        return cfg.lr * step / max(1, cfg.warmup)
    if step >= cfg.steps:
        return cfg.min_lr
    frac = (step - cfg.warmup) / max(1, cfg.steps - cfg.warmup)
    return cfg.min_lr + 0.5 * (1 + math.cos(math.pi * frac)) * (cfg.lr - cfg.min_lr)


def open_tokens(path: str) -> np.ndarray:
    if path.endswith(".npy"):
        return np.load(path, mmap_mode="r", allow_pickle=False)
    return np.memmap(path, dtype=np.uint16, mode="r")


class Batches:
    """Deterministic per-step batches: global batch ``s`` depends only on ``(seed, s)``."""

    def __init__(self, cfg: TrainConfig, rank: int, world: int, device: torch.device):
        self.cp = cfg.context_parallel and world > 1
        self.tp = cfg.tensor_parallel and world > 1  # every rank takes the whole batch
        if cfg.batch % world and not (self.cp or self.tp):
            raise ValueError(f"global batch {cfg.batch} must divide by world size {world}")
        self.world = world
        self.cfg, self.rank, self.local, self.device = cfg, rank, (cfg.batch if self.cp or self.tp else cfg.batch // world), device
        self.tokens = open_tokens(cfg.data) if cfg.data else None

    def __call__(self, step: int) -> tuple[torch.Tensor, torch.Tensor]:
        cfg = self.cfg
        g = torch.Generator().manual_seed(cfg.seed * 1_000_003 + step)
        # context parallel: every rank takes the whole batch and its part of each sequence
        lo, hi = (0, cfg.batch) if self.cp or self.tp else (self.rank * self.local, (self.rank + 1) * self.local)
        if self.tokens is None:
            toks = torch.randint(0, cfg.vocab, (cfg.batch, cfg.ctx + 1), generator=g)[lo:hi]
        else:
            starts = torch.randint(0, len(self.tokens) - cfg.ctx - 1, (cfg.batch,), generator=g)[lo:hi].numpy()
            idx = starts[:, None] + np.arange(cfg.ctx + 1)[None, :]
            toks = torch.from_numpy(np.asarray(self.tokens[idx]).astype(np.int64))
        if self.device.type == "cuda":
            toks = toks.pin_memory().to(self.device, non_blocking=True)
        x, y = toks[:, :-1].contiguous(), toks[:, 1:].contiguous()
        if self.cp:
            x = shard_sequence(x, self.rank, self.world, self.cfg.cp_layout)
            y = shard_sequence(y, self.rank, self.world, self.cfg.cp_layout)
        return x, y


def train(cfg: TrainConfig) -> dict:
    use_cuda = cfg.device == "cuda" or (cfg.device == "auto" and torch.cuda.is_available())
    rank, world, dev = setup_distributed(backend="nccl" if use_cuda else "gloo")
    torch.manual_seed(cfg.seed)
    model = build_model(cfg.size, cfg.ctx, vocab_size=cfg.vocab, device=dev)
    if cfg.context_parallel and world > 1:
        # sequence split over all ranks; gradients are still averaged over them by the DP wrapper
        enable_context_parallel(model, None, cfg.cp_layout)
    okw = dict(lr=cfg.lr, betas=(cfg.beta1, cfg.beta2), eps=cfg.eps, weight_decay=cfg.wd)
    shadows = dev.type == "cuda" and cfg.dtype == "bf16"
    zero = cfg.ddp == "zero"  # ZeRO-2: the wrapper owns the (sharded) optimizer, built after loading
    tp = cfg.tensor_parallel and world > 1  # TP: shard after loading the full weights, then build the optimizer
    if zero or tp or cfg.sharded:
        # ZeRO-1 is built after the DDP wrap: ShardedOptimizer re-homes every parameter into one flat
        # buffer per dtype, and DDPBucketed would then see the whole model as one storage unit (one
        # bucket, no overlap) if it were wrapped afterwards
        opt = None
    else:
        opt = ops.FusedAdamW(model.parameters(), bf16_shadows=shadows, **okw)

    start = 0
    path = latest_checkpoint(cfg.ckpt_dir) if cfg.resume and cfg.ckpt_dir else None
    if path is not None:
        meta = load_checkpoint(path, model, opt, map_location=dev)
        start = int(meta["step"])
        refresh_bf16_shadows(model.parameters())
        if rank == 0:
            print(f"resumed from {path} at step {start}", flush=True)
    # DDP wraps after loading so its initial broadcast ships the restored weights. A HIP-graph run
    # (single process) trains the bare model: the captured backward has no collectives to issue.
    use_graphs = cfg.graphs and world == 1 and dev.type == "cuda" and not zero
    if tp:
        tensor_parallel_(model)  # heads and d_ff over all ranks; no data-parallel wrapper
        opt = ops.FusedAdamW(model.parameters(), bf16_shadows=shadows, **okw)
        if path is not None:
            load_optimizer_state(path, opt, map_location=dev)
        ddp = model
    elif zero:
        ddp = ZeroDDP(model, bucket_size_mb=cfg.bucket_mb, bf16_shadows=shadows, **okw)
        opt = ddp.optimizer
        if path is not None:
            load_optimizer_state(path, opt, map_location=dev)
    else:
        ddp = model if use_graphs else wrap_ddp(model, cfg.ddp, bucket_size_mb=cfg.bucket_mb)
        if cfg.sharded:
            opt = ShardedOptimizer(model.parameters(), ops.FusedAdamW, bf16_shadows=shadows, **okw)
            if path is not None:
                load_optimizer_state(path, opt, map_location=dev)
    if isinstance(opt, ShardedOptimizer):
        opt.attach(ddp)  # the in-place parameter all-gather is waited for by the next forward
    graphed = None
    batches = Batches(cfg, rank, world, dev)
    amp = dev.type == "cuda" and cfg.dtype == "bf16"
    autocast = (lambda: torch.autocast("cuda", dtype=torch.bfloat16)) if amp else contextlib.nullcontext
    log = open(cfg.log_file, "a") if (cfg.log_file and rank == 0) else None
    hist = []
    t_last, tok_since = time.perf_counter(), 0
    loss_val = float("nan")
    end = min(cfg.steps, start + cfg.stop_after) if cfg.stop_after > 0 else cfg.steps
    for step in range(start, end):
        lr = lr_at(step, cfg)
        for g in opt.param_groups:
            g["lr"] = lr
        x, y = batches(step)
        if use_graphs:
            if graphed is None:
                from .utils.graphs import GraphedStep

                def loss_fn(xs, ys):
                    with autocast():
                        return ops.cross_entropy(model(xs), ys)

                graphed = GraphedStep(loss_fn, model.parameters(), x, y)
            loss = graphed(x, y)  # gradients land in the graph's static tensors, re-attached to .grad
        else:
            if hasattr(ddp, "zero_grad") and cfg.ddp in ("bucketed", "flat", "zero"):
                ddp.zero_grad()
            else:
                opt.zero_grad(set_to_none=True)
            with autocast():
                loss = ops.cross_entropy(ddp(x), y)
            loss.backward()
            if not tp:
                ddp.finish_gradient_synchronization()
        if cfg.clip > 0 and tp:
            gnorm = tp_clip_grad_norm_(model, cfg.clip)
        elif cfg.clip > 0:
            gnorm = ddp.clip_grad_norm_(cfg.clip) if zero else ops.clip_grad_norm_(model.parameters(), cfg.clip)
        else:
            gnorm = None
        opt.step()
        tok_since += cfg.batch * cfg.ctx
        done = step + 1
        if done % cfg.log_every == 0 or done == end:
            lt = loss.detach().float().clone()
            dist.all_reduce(lt)
            loss_val = float(lt) / world
            if not math.isfinite(loss_val):
                raise FloatingPointError(f"non-finite loss {loss_val} at step {done}; not checkpointing")
            if dev.type == "cuda":
                torch.cuda.synchronize(dev)
            now = time.perf_counter()
            rec = dict(step=done, loss=loss_val, lr=lr, tokens_per_s=tok_since / (now - t_last))
            if gnorm is not None:
                rec["grad_norm"] = float(gnorm)
            t_last, tok_since = now, 0
            hist.append(rec)
            if rank == 0:
                print(json.dumps(rec), flush=True)
                if log:
                    log.write(json.dumps(rec) + "\n")
                    log.flush()
        if cfg.ckpt_dir and ((cfg.ckpt_every and done % cfg.ckpt_every == 0) or done == end):
            if zero:
                ddp.wait_for_params()  # the parameter all-gathers of this step must land first
            elif isinstance(opt, ShardedOptimizer):
                opt.wait_parameters()
            # never let a diverged state become `latest` (keep-N would then prune the good ones):
            # this step's loss and the updated weights must be finite on every rank
            _check_finite_before_save(loss, model, done, dev)
            if tp:  # the full weights (gathered) and one optimizer file per rank
                save_checkpoint(cfg.ckpt_dir, done, model, opt, meta=dict(config=dataclasses.asdict(cfg)),
                                model_state=gather_tp_state_dict(model), sharded=True)
            else:
                save_checkpoint(cfg.ckpt_dir, done, model, opt, meta=dict(config=dataclasses.asdict(cfg)))
    if log:
        log.close()
    return dict(rank=rank, world=world, start=start, history=hist, final_loss=loss_val)


@torch.no_grad()
def _check_finite_before_save(loss: torch.Tensor, model: torch.nn.Module, step: int, dev: torch.device) -> None:
    """Raise on every rank if the loss or any (local) parameter is non-finite on any rank."""
    from .ops.adamw import multi_tensor_l2norm

    params = [p.detach() for p in model.parameters()]
    sq = multi_tensor_l2norm(params).float().reshape(1) if params else torch.zeros(1, device=dev)
    bad = (~torch.isfinite(loss.detach().float().reshape(1))) | (~torch.isfinite(sq))
    flag = bad.to(torch.float32).to(dev)
    if dist.is_initialized():
        dist.all_reduce(flag, op=dist.ReduceOp.MAX)
    if flag.item() > 0:
        raise FloatingPointError(f"non-finite loss or weights at step {step}; not checkpointing")


def parse(argv=None) -> TrainConfig:
    ap = argparse.ArgumentParser(description=__doc__.split("\n")[0])
    for f in dataclasses.fields(TrainConfig):
        name = "--" + f.name.replace("_", "-")
        if f.type in ("bool", bool):
            ap.add_argument(name, action="store_true", default=f.default)
        else:
            typ = {"int": int, "float": float}.get(str(f.type), str)
            ap.add_argument(name, type=typ, default=f.default)
    return TrainConfig(**vars(ap.parse_args(argv)))


def main(argv=None) -> int:
    cfg = parse(argv)
    try:
        train(cfg)
    finally:
        cleanup_distributed()
    return 0


if __name__ == "__main__":
    sys.exit(main())
