"""End-to-end model benchmarking and memory profiling (reference ``cs336_systems/benchmark.py``;
handout §1.1.3-1.1.6).

Per configuration it times, with device syncs at every boundary and HIP-event-free wall clocks
(the reference protocol, ``benchmark.py:91-117``):

* ``fwd``   — forward + loss,
* ``bwd``   — ``loss.backward()``,
* ``opt``   — ``optimizer.step()`` measured directly (the reference derived it as
  full − backward, reference bug 6),
* ``step``  — one complete training step (zero_grad → fwd → CE → bwd → step),

reports mean ± std, tokens/s and peak memory, and can dump a ``torch.cuda.memory`` snapshot of the
timed steps (viewable at pytorch.org/memory_viz). ``--compile`` really compiles (reference bug 6:
the flag was dropped).

    python -m cs336_systems.bench.e2e --sizes small medium large xl 2.7b --ctx 256 --batch 4 --mixed
    python -m cs336_systems.bench.e2e --memory --sizes 2.7b --ctx 128 256 512 --mixed
"""

from __future__ import annotations

import argparse
import contextlib
import json
import statistics
import time

import torch

from .. import ops
from ..data import synthetic_batch
from ..models import build_model, get_model_config, train_flops_per_token
from ..utils.memory import peak_mib, record_memory_history, reset_peak


def _sync(dev):
    if dev.type == "cuda":
        torch.cuda.synchronize(dev)


def _ms(f, dev):
    _sync(dev)
    t0 = time.perf_counter()
    out = f()
    _sync(dev)
    return (time.perf_counter() - t0) * 1e3, out


def run_simple_benchmark(
    size: str,
    context_length: int = 256,
    batch_size: int = 4,
    warmup_steps: int = 5,
    timed_steps: int = 10,
    mixed_precision: bool = False,
    compile: bool = False,
    device: str | None = None,
    vocab_size: int = 10000,
    optimizer: str = "fused",
    memory_snapshot: str | None = None,
    attention: str = "auto",
    graphs: bool = False,
) -> dict:
    from ..models import set_attention_impl

    dev = torch.device(device or ("cuda" if torch.cuda.is_available() else "cpu"))
    set_attention_impl(attention)
    torch.manual_seed(0)
    model = build_model(size, context_length, vocab_size=vocab_size, device=dev)
    if optimizer == "fused":
        opt = ops.FusedAdamW(model.parameters(), lr=1e-4, betas=(0.9, 0.95), eps=1e-8, weight_decay=0.01)
    else:
        from cs336_basics.optimizer import ReferenceAdamW

        opt = ReferenceAdamW(model.parameters(), lr=1e-4, betas=(0.9, 0.95), eps=1e-8, weight_decay=0.01)
    fmodel = torch.compile(model) if compile else model
    x, y = synthetic_batch(batch_size, context_length, vocab_size, dev)
    amp = mixed_precision and dev.type == "cuda"
    ctx = (lambda: torch.autocast(dev.type, dtype=torch.bfloat16)) if amp else contextlib.nullcontext

    def fwd():
        with ctx():
            return ops.cross_entropy(fmodel(x), y)

    def full():
        opt.zero_grad(set_to_none=True)
        loss = fwd()
        loss.backward()
        opt.step()
        return loss

    if graphs:
        # forward + loss + backward replayed from one HIP graph; AdamW runs eagerly after it
        from ..utils.graphs import GraphedStep

        def loss_fn(xs, ys):
            with ctx():
                return ops.cross_entropy(fmodel(xs), ys)

        gstep = GraphedStep(loss_fn, model.parameters(), x, y)

        def full():  # noqa: F811
            loss = gstep(x, y)
            opt.step()
            return loss

    for _ in range(warmup_steps):
        full()
    _sync(dev)
    reset_peak(dev)
    rec = {"fwd": [], "bwd": [], "opt": [], "step": []}
    with record_memory_history(memory_snapshot):
        for _ in range(0 if graphs else timed_steps):  # a graph replays fwd+bwd as one unit
            opt.zero_grad(set_to_none=True)
            t, loss = _ms(fwd, dev)
            rec["fwd"].append(t)
            t, _ = _ms(loss.backward, dev)
            rec["bwd"].append(t)
            t, _ = _ms(opt.step, dev)
            rec["opt"].append(t)
        for _ in range(timed_steps):
            t, _ = _ms(full, dev)
            rec["step"].append(t)
    out = dict(size=size, ctx=context_length, batch=batch_size, mixed=mixed_precision, compile=compile, attention=attention, graphs=graphs)
    for k, v in rec.items():
        out[f"{k}_ms"] = statistics.fmean(v) if v else float("nan")
        out[f"{k}_std"] = statistics.pstdev(v) if len(v) > 1 else 0.0
    toks = batch_size * context_length
    out["tokens_per_s"] = toks / (out["step_ms"] / 1e3)
    out["model_tflops"] = out["tokens_per_s"] * train_flops_per_token(size, context_length, vocab_size) / 1e12
    out["peak_mib"] = peak_mib(dev)
    return out


def run_memory_profile(size: str, context_length: int, mode: str = "fullstep", mixed_precision: bool = True, batch_size: int = 4, snapshot: str | None = None, device=None) -> float:
    """Peak memory (MiB) of a forward-only pass or a full training step (reference ``:175-245``)."""
    dev = torch.device(device or "cuda")
    torch.manual_seed(0)
    model = build_model(size, context_length, device=dev)
    opt = ops.FusedAdamW(model.parameters(), lr=1e-4)
    x, y = synthetic_batch(batch_size, context_length, 10000, dev)
    ctx = torch.autocast(dev.type, dtype=torch.bfloat16) if mixed_precision else contextlib.nullcontext()
    reset_peak(dev)
    with record_memory_history(snapshot):
        if mode == "forward":
            # grad mode on, as in the reference: the live logits keep every saved activation
            with ctx:
                logits = model(x)
            del logits
        else:
            with ctx:
                loss = ops.cross_entropy(model(x), y)
            loss.backward()
            opt.step()
        _sync(dev)
    return peak_mib(dev)


def _table(rows: list[dict], cols: list[str]) -> str:
    try:
        import pandas as pd

        return pd.DataFrame(rows)[cols].to_markdown(index=False, floatfmt=".2f")
    except Exception:
        head = "| " + " | ".join(cols) + " |\n|" + "---|" * len(cols) + "\n"
        return head + "\n".join("| " + " | ".join(f"{r.get(c, ''):.2f}" if isinstance(r.get(c), float) else str(r.get(c, "")) for c in cols) + " |" for r in rows)


def main(argv=None):
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--sizes", nargs="+", default=["small"])
    ap.add_argument("--ctx", nargs="+", type=int, default=[256])
    ap.add_argument("--batch", type=int, default=4)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--mixed", action="store_true")
    ap.add_argument("--compile", action="store_true")
    ap.add_argument("--graphs", action="store_true", help="replay forward+backward from one captured HIP graph")
    ap.add_argument("--optimizer", default="fused", choices=["fused", "reference"])
    ap.add_argument("--attention", default="auto", choices=["auto", "naive", "flash"])
    ap.add_argument("--memory", action="store_true", help="memory profile (forward and fullstep) instead of timing")
    ap.add_argument("--snapshot-dir", default=None)
    ap.add_argument("--json", default=None)
    a = ap.parse_args(argv)
    rows = []
    for size in a.sizes:
        for ctx in a.ctx:
            try:
                if a.memory:
                    for mode in ("forward", "fullstep"):
                        snap = None
                        if a.snapshot_dir:
                            snap = f"{a.snapshot_dir}/memory_{size}_ctx{ctx}_{mode}_{'mixed' if a.mixed else 'fp32'}.pickle"
                        rows.append(dict(size=size, ctx=ctx, mode=mode, mixed=a.mixed, peak_mib=run_memory_profile(size, ctx, mode, a.mixed, a.batch, snap)))
                else:
                    rows.append(run_simple_benchmark(size, ctx, a.batch, a.warmup, a.steps, a.mixed, a.compile, optimizer=a.optimizer, attention=a.attention, graphs=a.graphs))
            except torch.OutOfMemoryError:
                rows.append(dict(size=size, ctx=ctx, error="OOM"))
            torch.cuda.empty_cache() if torch.cuda.is_available() else None
            print(json.dumps(rows[-1]), flush=True)
    cols = ["size", "ctx", "mode", "mixed", "peak_mib"] if a.memory else ["size", "ctx", "mixed", "fwd_ms", "fwd_std", "bwd_ms", "bwd_std", "opt_ms", "step_ms", "step_std", "tokens_per_s", "model_tflops", "peak_mib"]
    print(_table([r for r in rows if "error" not in r], cols))
    if a.json:
        with open(a.json, "w") as f:
            json.dump(rows, f, indent=1)


if __name__ == "__main__":
    main()
