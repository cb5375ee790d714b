#!/usr/bin/env python
"""Headline benchmark: GPT-2-XL-shape Transformer LM, bf16 mixed-precision full training step,
data-parallel over RCCL/xGMI, tokens/s for the whole node (BASELINE.json metric/config).

    python bench.py --gpus 1 --steps 10 --warmup 3
    python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 \
        --master-port 29500 bench.py --gpus 8 --steps 10 --warmup 3

One step = zero grads → forward (bf16 autocast over fp32 master weights; HIP RMSNorm/RoPE/
FlashAttention-2 kernels, cs336 MFMA GEMMs with the SwiGLU / RoPE epilogues fused, per-problem
table against hipBLASLt) → fused HIP cross-entropy → backward with the bucketed DDP all-reduce
overlapped (N > 1) → fused multi-tensor HIP AdamW on all 2.0 B params (on one GPU launched chunk
by chunk during the backward, as gradients become final).
Model "xl" = d_model 1600, 48 layers, 25 heads (d_head 64), d_ff 6400, vocab 10000, ctx 512
(reference ``cs336_systems/benchmark.py:247-259``), random init, synthetic tokens.
Weak scaling: the per-GPU batch is fixed, so global batch = batch * N.
Timing: W untimed warmup steps, then barrier + synchronize, K steps, synchronize + barrier;
the slowest rank's wall time is reported (MAX over ranks).
"""

from __future__ import annotations

import argparse
import json
import os
import socket
import subprocess
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

from cs336_systems.rccl_env import apply_multi_gpu_env  # noqa: E402  (torch-free)

if __name__ == "__main__":
    # stream-K grid cap for multi-rank runs (the RCCL channel cap was dropped in round 4; the cap is
    # inert on this image and kept for hipBLASLt builds that honour it), set before torch loads
    # hipBLASLt/RCCL (cs336_systems/rccl_env.py, profiles/r4_streamk_cap.md)
    _CORES_ENV = apply_multi_gpu_env(int(os.environ.get("WORLD_SIZE", "1")))
else:
    _CORES_ENV = {}

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

METRIC = "tokens/sec/node GPT-2-XL bf16 DDP"
BASELINE_VALUE = None  # the reference publishes no number


def emit_result(out: dict, json_out: str | None) -> None:
    """The ONE JSON result line (rank 0), also written to ``--json-out``."""
    line = json.dumps(out)
    print(line, flush=True)
    if json_out:
        with open(json_out, "w") as f:
            f.write(line + "\n")


class SweepWatchdog:
    """Bounds the post-headline DDP sweep. The headline fields are final before the sweep starts; if a
    variant stalls (a collective that never completes would otherwise sit until the process group's
    600 s timeout aborts the job without a result line), the timer marks the sweep timed out, rank 0
    prints the headline line, and every rank leaves with status 0 (``os._exit``: the main thread is
    blocked in the stuck call). Each rank arms its own timer, so no collective is needed to stop."""

    def __init__(self, out: dict, rank: int, json_out: str | None, limit_s: float):
        import threading

        self.out, self.rank, self.json_out, self.limit_s = out, rank, json_out, limit_s
        self._lock = threading.Lock()
        self._done = False
        self._timer = threading.Timer(limit_s, self._fire)
        self._timer.daemon = True
        self._timer.start()

    def cancel(self) -> None:
        with self._lock:
            self._done = True
        self._timer.cancel()

    def _fire(self) -> None:
        with self._lock:
            if self._done:
                return
            self._done = True
        self.out.setdefault("dist", {})["ddp_sweep"] = {"error": f"timed out after {self.limit_s:g} s",
                                                        "watchdog": True}
        if self.rank == 0:
            log(f"DDP sweep exceeded {self.limit_s:g} s: reporting the headline result without it")
            emit_result(self.out, self.json_out)
        sys.stderr.flush()
        os._exit(0)


def log(*a):
    if int(os.environ.get("RANK", "0")) == 0:
        print(*a, file=sys.stderr, flush=True)


def parse(argv=None):
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--model", default="xl")
    ap.add_argument("--ctx", type=int, default=512)
    # 102 x 512 = 52224 tokens per GPU (198 GiB of the 288): 204 row tiles of 256, so every d_model-wide
    # projection output (N 1600 = 5 tiles of 320) fills 1020 of 4 x 256 CU slots instead of 960 at batch
    # 96 (3.75 rounds, the last a quarter idle). Same box, 2 rounds: 96 -> 87.5-87.6k, 100 -> 88.2k,
    # 102 -> 88.6k tok/s (profiles/r5_batch102.md; GEMM table and dW plans cover 52224 tokens).
    # Earlier: 96 x 512 = 49152 tokens per GPU (188 GiB of the 288). Per-GPU batch sweep of the XL step on
    # 1x MI355X with the round-3 kernels (profiles/r3_batch_sweep_s5.md): 48 -> 83.5k, 72 -> 84.3k,
    # 96 -> 85.9-86.1k tok/s -- the per-step fixed costs (fused AdamW over 2.0 B parameters, the
    # vocabulary head, launch tails) amortize over twice the tokens, and under DDP the backward that
    # hides each step's 8 GB gradient all-reduce doubles. (Round 2, hipBLASLt-era sweep:
    # profiles/r2_batch_sweep.md.) The committed GEMM table and dW plans cover 24576 and 49152 tokens.
    # (2.7b: 32 x 1024 = 32768 tokens per GPU by default, 164 GiB: 53.2-53.4k tok/s vs 51.6k at 24 x 1024
    # (136 GiB) and 45.6k at 12 x 1024, where every d_model-wide GEMM output has only 384 tiles of
    # 256 x 320 for 256 CUs; profiles/r4_bench_2p7b.md, the committed table covers 12288, 24576 and
    # 32768 tokens)
    ap.add_argument("--batch", type=int, default=None, help="per-GPU batch (default: xl 102, 2.7b 32768 tokens / ctx)")
    ap.add_argument("--vocab", type=int, default=10000)
    ap.add_argument(
        "--ddp",
        default="bucketed",
        choices=["bucketed", "individual", "flat", "naive", "zero"],
        help="zero = ZeRO-2: reduce-scattered grads, sharded fused AdamW, param all-gather under the next forward",
    )
    ap.add_argument("--bucket-mb", type=float, default=None)
    ap.add_argument(
        "--grad-comm-dtype",
        default="fp32",
        choices=["fp32", "bf16"],
        help="bucketed DDP / ZeRO-2: dtype of the gradients on the wire (bf16 halves the all-reduce / reduce-scatter bytes)",
    )
    ap.add_argument("--sharded", action="store_true", help="ZeRO-1 sharded optimizer state")
    ap.add_argument("--ddp-world1", action="store_true",
                    help="diagnostic: wrap the model in --ddp over a one-rank RCCL group at N = 1 (DDP's own cost)")
    ap.add_argument("--dtype", default="bf16", choices=["bf16", "fp32"])
    ap.add_argument("--lr", type=float, default=1e-4)
    ap.add_argument("--clip", type=float, default=0.0, help="global grad-norm clip (0 = off, as the reference bench)")
    ap.add_argument("--backend", default=os.environ.get("CS336_BACKEND", "auto"))
    ap.add_argument("--json-out", default=None)
    ap.add_argument("--no-shadows", action="store_true", help="autocast re-casts weights every forward (A/B)")
    ap.add_argument("--no-fused-layout", action="store_true", help="separate q/k/v and w1/w3 GEMMs (A/B)")
    ap.add_argument(
        "--overlap-opt",
        default="auto",
        choices=["auto", "on", "off"],
        # XL at batch 102 (round 5, same box, 3 rounds): 576.7 / 577.1 / 577.3 ms/step overlapped vs
        # 580.8 / 580.9 / 582.6 off (profiles/r5_opt_overlap_ab.md): the HBM-bound update of each
        # layer's weights runs beside the next layers' backward. (Round 1, batch 24 and the older
        # kernels: 193.0 on vs 189.2 off.) Bitwise the same update (tests/test_opt_overlap_gpu.py)
        help="run the AdamW update during backward on a side stream (auto: on a single GPU when clip == 0 and not sharded)",
    )
    ap.add_argument(
        "--gemm",
        default=os.environ.get("CS336_GEMM", "best"),
        choices=["blas", "lt", "best", "hip"],
        # same-box A/B at batch 48 (profiles/r2_batch_sweep.md): blas 354.1/355.0 ms/step, lt 340.6/342.9,
        # best 331.4/332.2 (the autotuned / cs336 picks win on W1|W3 dX, the o-projection and lm_head)
        help="projection GEMM selection (cs336_systems/ops/gemm.py); sets CS336_GEMM",
    )
    ap.add_argument(
        "--graphs",
        default="off",
        choices=["on", "off"],
        help="1 GPU: capture the WHOLE step (zero grads, forward, loss, backward, AdamW -- overlapped or not) once "
        "into a HIP graph and replay it every step (utils/graphs.py GraphedTrainStep; device-side AdamW step counter)",
    )
    ap.add_argument(
        "--comm-sweep-mb",
        type=float,
        nargs="*",
        default=[1, 10, 100, 1024],
        help="N > 1: after the timed steps, fp32 all-reduce sweep (5 warmup + 5 timed each) added to the JSON's dist block",
    )
    ap.add_argument(
        "--ddp-sweep",
        default="auto",
        choices=["auto", "on", "off"],
        help="N > 1 (auto: with RCCL): after the timed steps, the handout's DDP comparison -- naive / flat / "
        "per-parameter / bucketed {1,10,100,1000} MB ms/step + comm wait, ZeRO-1 memory -- into the JSON's dist "
        "block (<= 60 s)",
    )
    ap.add_argument("--ddp-sweep-batch", type=int, default=4, help="per-GPU batch of the DDP sweep")
    ap.add_argument(
        "--ddp-sweep-timeout",
        type=float,
        default=240.0,
        help="wall-clock limit of the DDP sweep: past it every rank stops, rank 0 having printed the headline line "
        "with the sweep marked timed out (a stuck collective never costs the headline result)",
    )
    ap.add_argument(
        "--tunableop",
        default="auto",
        choices=["auto", "off", "use", "tune"],
        help="PyTorch TunableOp GEMM selection: use = load committed hipBLASLt/rocBLAS picks, tune = re-tune and save",
    )
    a = ap.parse_args(argv)
    if a.batch is None:
        env = os.environ.get("CS336_BENCH_BATCH")
        a.batch = int(env) if env else (max(1, 32768 // a.ctx) if a.model == "2.7b" else 102)
    return a


def setup_tunableop(mode: str, rank: int) -> str | None:
    """Per-shape GEMM solution selection (hipBLASLt vs rocBLAS candidates), tuned once on MI355X and
    committed under cs336_systems/tuning/ so every fresh box replays the same picks."""
    from cs336_systems.tuning import tunableop_file

    path = tunableop_file()
    if mode == "auto":
        mode = "use" if os.path.exists(path) else "off"
    if mode == "off":
        return None
    import torch.cuda.tunable as tunable

    tunable.enable(True)
    tunable.set_max_tuning_duration(50)
    tunable.set_max_tuning_iterations(60)
    if mode == "tune":
        tunable.tuning_enable(True)
        tunable.set_filename(path + (f".rank{rank}" if rank else ""))
    else:
        tunable.tuning_enable(False)
        tunable.read_file(path)
    log(f"TunableOp: {mode} ({path})")
    return mode


def self_launch(n: int, argv: list[str]) -> int:
    """``python bench.py --gpus N`` without a launcher: run the same command under
    ``torch.distributed.run`` with N ranks on this node (127.0.0.1 rendezvous) and return its exit
    code. Called before anything touches the GPU; the ranks are child processes (no exec)."""
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", f"--master-port={port}", os.path.abspath(__file__), *argv]
    log(f"bench.py --gpus {n} without WORLD_SIZE: launching {n} ranks: {' '.join(cmd)}")
    return subprocess.call(cmd)


def comm_sweep(sizes_mb, device, world) -> list[dict]:
    """The reference's all-reduce microbenchmark (``distributed_communication_single.py:28-148``,
    handout p.26: fp32, 5 warmup + timed calls) on the job's own process group, after the timed
    steps: per size the max over ranks of the mean time, algorithm and bus bandwidth."""
    from cs336_systems.bench.collectives import _busbw_factor, run_collective

    rows = []
    for mb in sizes_mb:
        nbytes = int(mb * 2**20)
        t = run_collective("all_reduce", nbytes, device, warmup=5, iters=5)
        on_dev = dist.get_backend() == "nccl"
        tt = torch.tensor([t], dtype=torch.float64, device=device if on_dev else "cpu")
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        t = float(tt.item())
        algbw = nbytes / t / 1e9
        rows.append({"size_mb": mb, "ms": round(t * 1e3, 4), "algbw_gbs": round(algbw, 3),
                     "busbw_gbs": round(algbw * _busbw_factor("all_reduce", world), 3)})
        if device.type == "cuda":
            torch.cuda.empty_cache()
    return rows


def dist_diagnostics(ddp_model, comm_wait_ms, device, world) -> dict:
    """What a multi-GPU run needs to be diagnosable from its own JSON line: exposed communication
    per step (max over ranks), the bucket layout, the process group as the ranks see it, the
    RCCL version and environment, and a standalone all-reduce of the largest bucket (bus bandwidth
    without compute beside it)."""
    d: dict = {"pg_world_size": dist.get_world_size(), "backend": dist.get_backend()}
    if comm_wait_ms is not None:
        on_dev = dist.get_backend() == "nccl"
        t = torch.tensor([comm_wait_ms], dtype=torch.float64, device=device if on_dev else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        d["comm_wait_ms"] = round(float(t.item()), 3)
    buckets = ddp_model.bucket_summary() if hasattr(ddp_model, "bucket_summary") else []
    if buckets:
        mbs = [b["mb"] for b in buckets]
        d["n_buckets"] = len(mbs)
        d["bucket_mb"] = {"min": round(min(mbs), 2), "max": round(max(mbs), 2), "total": round(sum(mbs), 1)}
        d["bucket_sizes_mb"] = [round(m, 1) for m in mbs]
        if "wire_mb" in buckets[0]:
            d["wire_dtype"] = buckets[0]["wire"]
            d["wire_mb_total"] = round(sum(b["wire_mb"] for b in buckets), 1)
    try:
        v = torch.cuda.nccl.version()
        d["rccl_version"] = ".".join(map(str, v)) if isinstance(v, tuple) else str(v)
    except Exception as e:  # noqa: BLE001 - diagnostic only
        d["rccl_version"] = f"unavailable ({type(e).__name__})"
    d["env"] = {k: v for k, v in sorted(os.environ.items())
                if k.startswith(("NCCL_", "RCCL_", "HSA_", "TORCH_NCCL_", "TENSILE_STREAMK"))}
    d["coresidency_caps"] = dict(_CORES_ENV)
    # per-rank CPU affinity (each rank pinned to its GPU's NUMA-local CPUs in setup_distributed)
    from cs336_systems.parallel.affinity import affinity_info

    per_rank: list = [None] * dist.get_world_size()
    dist.all_gather_object(per_rank, {"rank": dist.get_rank(), **affinity_info()})
    d["cpu_affinity"] = per_rank
    if buckets and world > 1 and device.type == "cuda" and dist.get_backend() == "nccl":
        n = int(max(mbs) * 2**20 // 4)
        buf = torch.ones(n, dtype=torch.float32, device=device)
        for _ in range(2):
            dist.all_reduce(buf)
        torch.cuda.synchronize(device)
        reps = 5
        t0 = time.perf_counter()
        for _ in range(reps):
            dist.all_reduce(buf)
        torch.cuda.synchronize(device)
        dt = (time.perf_counter() - t0) / reps
        algbw = n * 4 / dt / 1e9
        d["allreduce_probe"] = {"mb": round(n * 4 / 2**20, 1), "ms": round(dt * 1e3, 3), "algbw_gbs": round(algbw, 1),
                                "busbw_gbs": round(algbw * 2 * (world - 1) / world, 1)}
        del buf
    return d


def main(argv=None):
    argv = list(sys.argv[1:] if argv is None else argv)
    args = parse(argv)
    world_env = os.environ.get("WORLD_SIZE")
    if world_env is None and args.gpus > 1:
        return self_launch(args.gpus, argv)  # never a mislabeled 1-GPU number
    world = int(world_env or 1)
    if world != args.gpus:
        log(f"error: --gpus {args.gpus} but WORLD_SIZE={world} (launch N ranks for --gpus N)")
        return 2
    rank = int(os.environ.get("RANK", "0"))

    os.environ["CS336_GEMM"] = args.gemm  # read per call by cs336_systems.ops.gemm
    from cs336_systems import ops
    from cs336_systems.data import synthetic_batch
    from cs336_systems.models import build_model, get_model_config, param_count, train_flops_per_token
    from cs336_systems.parallel import DEFAULT_BUCKET_MB, ShardedOptimizer, ZeroDDP, setup_distributed, wrap_ddp

    ops.set_backend(args.backend)
    zero = args.ddp == "zero"
    dist_on = world > 1 or zero or args.ddp_world1
    if dist_on:  # (zero / --ddp-world1 at world 1: a one-rank group, to measure the wrapper's overhead)
        # CS336_DIST_BACKEND=gloo: rehearse the multi-rank path with several ranks on one GPU
        rank, world, device = setup_distributed(
            backend=os.environ.get("CS336_DIST_BACKEND") or None, use_gpu=torch.cuda.is_available()
        )
    else:
        device = torch.device("cuda", 0) if torch.cuda.is_available() else torch.device("cpu")
        if device.type == "cuda":
            torch.cuda.set_device(device)
            # the host threads on the CPUs local to the GPU, as every rank of a multi-GPU run is
            # (setup_distributed): the eager step's launch stream runs from them
            # (neutral on one GPU, 585.8-586.0 vs 586.0-586.4 ms: profiles/r6_ddp_world1.md)
            from cs336_systems.parallel.affinity import pin_rank_to_gpu

            pin_rank_to_gpu(device)
    tmode = None
    if device.type == "cuda":
        assert ops.ext_available(), ops.load_error()
        torch.backends.cuda.matmul.allow_tf32 = False
        tmode = setup_tunableop(args.tunableop, rank)

    torch.manual_seed(1234)
    t0 = time.time()
    model = build_model(args.model, args.ctx, vocab_size=args.vocab, device=device, fused_layout=not args.no_fused_layout)
    n_params = sum(p.numel() for p in model.parameters())
    log(f"built {args.model}: {n_params / 1e9:.3f} B params in {time.time() - t0:.1f}s on {device}")

    amp = args.dtype == "bf16" and device.type == "cuda"
    okw = dict(lr=args.lr, betas=(0.9, 0.95), eps=1e-8, weight_decay=0.01)
    # bf16 compute-weight shadows written by the AdamW kernel (models/fused.py)
    shadows = amp and not args.no_shadows
    bucket = args.bucket_mb if args.bucket_mb is not None else DEFAULT_BUCKET_MB
    if zero:
        zkw = {"comm_dtype": torch.bfloat16} if args.grad_comm_dtype == "bf16" else {}
        ddp_model = ZeroDDP(model, bucket_size_mb=bucket, bf16_shadows=shadows, **zkw, **okw)
    elif world > 1 or args.ddp_world1:
        kw = {"comm_dtype": torch.bfloat16} if args.grad_comm_dtype == "bf16" and args.ddp == "bucketed" else {}
        ddp_model = wrap_ddp(model, args.ddp, bucket_size_mb=bucket, **kw)
    else:
        ddp_model = model
    # auto: without a process group only. Beside RCCL's collectives the update also competes for the
    # CUs and HBM the bucket all-reduces use: with the W = 8 ring's bytes emulated beside the real XL
    # backward the overlapped update is slower in five of six bucket / channel configurations (+5.6 to
    # +63.5 ms; 128 MB, 32 channels: 635.0 vs 629.4 ms, profiles/r6_comm_emulation.md), and under the
    # one-rank DDP wrapper 608.3 / 609.1 ms on vs 606.6 / 605.5 off (profiles/r5_opt_overlap_ab.md)
    use_graphs = args.graphs == "on" and world == 1 and device.type == "cuda" and not dist_on and args.clip == 0
    overlap = args.overlap_opt == "on" or (
        args.overlap_opt == "auto" and device.type == "cuda" and args.clip == 0 and not args.sharded and not dist_on
    )
    if zero:
        opt = ddp_model.optimizer
        overlap = False
    elif args.sharded and world > 1:
        # in-place async parameter all-gather, waited for by the next forward (stream dependency)
        opt = ShardedOptimizer(model.parameters(), ops.FusedAdamW, bf16_shadows=shadows, **okw).attach(ddp_model)
        overlap = False
    else:
        opt = ops.FusedAdamW(model.parameters(), bf16_shadows=shadows, **okw)
        if overlap:
            # the update of each parameter (DDP: each reduced bucket) runs during backward
            overlap = opt.enable_backward_overlap(ddp=ddp_model if ddp_model is not model else None)

    gen = torch.Generator(device=device)
    gen.manual_seed(1000 + rank)
    batches = [synthetic_batch(args.batch, args.ctx, args.vocab, device, gen) for _ in range(4)]

    def zero_grads():
        # unset grads: the projection GEMMs then write fp32 dW straight into the DDP buckets
        opt.zero_grad(set_to_none=True)

    def eager_step(x, y):
        """One complete step on the current stream (also what GraphedTrainStep captures)."""
        zero_grads()
        with torch.autocast(device.type, dtype=torch.bfloat16, enabled=amp):
            logits = ddp_model(x)
            loss = ops.cross_entropy(logits, y)
        loss.backward()
        opt.step()
        # detached: a loss that keeps its autograd graph alive also keeps the parameters' AccumulateGrad
        # nodes (bound to the stream of their first backward), which breaks a later capture on a side stream
        return loss.detach()

    graphed = None

    # exposed communication: GPU time the compute stream spends waiting in
    # finish_gradient_synchronization for collectives that backward did not hide (HIP events)
    comm_events: list[tuple] = []
    timing = {"on": False}

    def step(i):
        x, y = batches[i % len(batches)]
        if graphed is not None:  # the whole captured step, AdamW included
            return graphed(x, y)
        zero_grads()
        with torch.autocast(device.type, dtype=torch.bfloat16, enabled=amp):
            logits = ddp_model(x)
            loss = ops.cross_entropy(logits, y)
        loss.backward()
        if dist_on:
            if timing["on"] and device.type == "cuda":
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                ddp_model.finish_gradient_synchronization()
                e1.record()
                comm_events.append((e0, e1))
            elif timing["on"]:  # CPU/gloo: the wait blocks the host
                t0 = time.perf_counter()
                ddp_model.finish_gradient_synchronization()
                comm_events.append(1e3 * (time.perf_counter() - t0))
            else:
                ddp_model.finish_gradient_synchronization()
        if args.clip > 0 and zero:
            ddp_model.clip_grad_norm_(args.clip)
        elif args.clip > 0:
            ops.clip_grad_norm_(model.parameters(), args.clip)
        opt.step()
        return loss.detach()

    def sync():
        if device.type == "cuda":
            torch.cuda.synchronize(device)

    def barrier():
        if world > 1:
            dist.barrier()

    # lt/best GEMM modes time their candidates the first time each problem shape is seen: with
    # --warmup 0 one untimed step still runs so that selection never lands inside the timed region
    n_warm = max(args.warmup, 1) if device.type == "cuda" and args.gemm in ("lt", "best") else args.warmup
    if use_graphs:
        # two real steps before the capture: one eager (optimizer state, GEMM selection) and one on the
        # capture stream inside GraphedTrainStep; the rest of the warmup replays the graph
        n_warm = max(n_warm, 2)
    for i in range(n_warm):
        if use_graphs and i == 1:
            from cs336_systems.utils.graphs import GraphedTrainStep

            t0 = time.time()
            graphed = GraphedTrainStep(eager_step, opt, *batches[i % len(batches)], warmup=1)
            loss = graphed.warmup_loss
            log(f"captured the whole step into one HIP graph in {time.time() - t0:.1f}s")
        else:
            loss = step(i)
        sync()
        log(f"warmup {i}: loss {loss.item():.4f}")
    if device.type == "cuda":
        torch.cuda.reset_peak_memory_stats(device)
    barrier()
    sync()
    timing["on"] = True
    from cs336_systems.utils.gpu_monitor import GpuSampler

    # clock / power / temperature over the timed window (the JSON's gpu_clocks block): explains a
    # box-to-box spread of the same tree (DVFS under the MFMA-dense step)
    sampler = GpuSampler(device)
    ms0 = torch.cuda.memory_stats(device) if device.type == "cuda" else {}
    t_start = time.perf_counter()
    sync_each = os.environ.get("CS336_BENCH_SYNC_EACH", "0") == "1"  # diagnostic: no host run-ahead
    with sampler:
        for i in range(args.steps):
            loss = step(i)
            if sync_each:
                sync()
        sync()
    barrier()
    elapsed = time.perf_counter() - t_start
    timing["on"] = False
    last_loss = loss.item()
    comm_wait_ms = (
        sum(e if isinstance(e, float) else e[0].elapsed_time(e[1]) for e in comm_events) / len(comm_events)
        if comm_events
        else None
    )
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=device)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    peak_gib = torch.cuda.max_memory_allocated(device) / 2**30 if device.type == "cuda" else 0.0
    if device.type == "cuda":  # allocator churn inside the timed steps (cudaFree/cudaMalloc retries)
        ms = torch.cuda.memory_stats(device)
        log(
            f"allocator: reserved peak {ms.get('reserved_bytes.all.peak', 0) / 2**30:.1f} GiB, "
            f"alloc retries {ms.get('num_alloc_retries', 0)}, device mallocs {ms.get('num_device_alloc', 0)}"
        )
        alloc_timed = {k: ms.get(k, 0) - ms0.get(k, 0) for k in
                       ("num_device_alloc", "num_device_free", "num_sync_all_streams", "num_alloc_retries")}

    ms_per_step = 1e3 * elapsed / max(args.steps, 1)
    tokens_per_step = args.batch * args.ctx * world
    value = tokens_per_step * args.steps / elapsed
    flops_tok = train_flops_per_token(args.model, args.ctx, args.vocab)
    mfu = value * flops_tok / (world * 2.5e15)
    cfg = get_model_config(args.model)
    out = {
        "metric": METRIC if args.model == "xl" else METRIC.replace("GPT-2-XL", f"{args.model} (not the headline model)"),
        "value": round(value, 1),
        "unit": "tokens/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(ms_per_step, 2),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": (value / BASELINE_VALUE) if BASELINE_VALUE else None,
        "dtype": "bf16" if amp else "fp32",
        "data": "synthetic (random tokens on device, random-init weights)",
        "config": {
            "model": f"{args.model} ({'GPT-2-XL shape: ' if args.model == 'xl' else ''}d_model {cfg['d_model']}, {cfg['num_layers']} layers, {cfg['num_heads']} heads, d_ff {cfg['d_ff']}, vocab {args.vocab}, {param_count(args.model, args.vocab) / 1e9:.2f}B params)",
            "global_batch": args.batch * world,
            "per_gpu_batch": args.batch,
            "seq_len": args.ctx,
            "parallelism": f"dp{world}" + ("+zero2" if zero else "+zero1" if args.sharded and world > 1 else ""),
            "ddp": args.ddp if dist_on else "none",
            "bucket_mb": bucket if dist_on else None,
            "grad_comm_dtype": args.grad_comm_dtype if world > 1 and (args.ddp == "bucketed" or zero) else None,
            "optimizer": "fused HIP AdamW (fp32 master weights)"
            + (", overlapped with backward" if overlap else "")
            + (", sharded 1/W with param all-gather under the forward" if zero else ""),
            "attention": "HIP FlashAttention-2 (causal)",
            "hip_graph": graphed is not None,
        },
        "mfu_dense_bf16": round(mfu, 4),
        "model_tflops_per_gpu": round(value * flops_tok / world / 1e12, 1),
        "peak_mem_gib": round(peak_gib, 2),
        "final_loss": round(last_loss, 4),
        "gpu_clocks": sampler.summary(),
    }
    if device.type == "cuda":  # caching-allocator events inside the timed steps (hipMalloc/hipFree sync)
        out["allocator_timed"] = alloc_timed
    if device.type == "cuda" and not dist_on:
        from cs336_systems.parallel.affinity import affinity_info

        out["cpu_affinity"] = affinity_info()
    if device.type != "cuda":  # CPU rehearsal: eager PyTorch reference ops, no HIP kernels ran
        out["config"]["optimizer"] = out["config"]["optimizer"].replace("fused HIP AdamW", "PyTorch-reference AdamW")
        out["config"]["attention"] = "PyTorch-reference attention (causal)"
    from cs336_systems.ops.gemm import _mode as gemm_mode

    gsel = {"blas": "hipblaslt default", "lt": "autotuned hipblaslt (cs336 lt_gemm)",
            "best": "per-problem fastest of hipblaslt default / autotuned lt_gemm / cs336 MFMA GEMM", "hip": "cs336 MFMA GEMM"}[gemm_mode()]
    out["config"]["gemm_selection"] = f"tunableop:{tmode}" if tmode else gsel if device.type == "cuda" else "torch cpu"
    if dist_on:
        out["dist"] = dist_diagnostics(ddp_model, comm_wait_ms, device, world)
        if world > 1 and args.comm_sweep_mb:
            out["dist"]["allreduce_sweep_fp32"] = comm_sweep(args.comm_sweep_mb, device, world)
    # auto: with RCCL (the driver's multi-GPU runs); a gloo rehearsal stages every all-reduce through
    # the host (minutes per variant at XL), so there it runs only when asked for (--ddp-sweep on)
    run_sweep = args.ddp_sweep == "on" or (args.ddp_sweep == "auto" and dist.is_initialized()
                                            and dist.get_backend() == "nccl")
    if world > 1 and run_sweep and not zero:
        # the headline fields are final; free the timed model, then the bounded DDP-variant table
        del ddp_model, opt, model, batches, graphed, eager_step
        if device.type == "cuda":
            torch.cuda.empty_cache()
        from cs336_systems.bench.ddp import sweep_variants

        # the sweep's small per-GPU batch has no committed GEMM-table entries; in a multi-rank job those
        # would run hipBLASLt's stream-K default beside the RCCL all-reduces (rccl_env.py), so the sweep
        # uses the cs336 kernels only (gemm8 / gemm8w take every projection shape of it)
        gemm_mode_saved = os.environ.get("CS336_GEMM")
        os.environ["CS336_GEMM"] = "hip" if device.type == "cuda" else gemm_mode_saved or "blas"
        dog = SweepWatchdog(out, rank, args.json_out, args.ddp_sweep_timeout)
        try:
            sw = sweep_variants(args.model, args.ctx, args.ddp_sweep_batch, device, amp=amp, vocab=args.vocab)
            dog.cancel()
            out["dist"]["ddp_variants"] = sw.pop("variants")
            out["dist"]["zero1_memory"] = sw.pop("zero1_memory")
            out["dist"]["ddp_sweep"] = sw
        except Exception as e:  # noqa: BLE001 - the sweep never costs the headline line
            dog.cancel()
            out["dist"]["ddp_sweep"] = {"error": f"{type(e).__name__}: {e}"[:300]}
        finally:
            if gemm_mode_saved is None:
                os.environ.pop("CS336_GEMM", None)
            else:
                os.environ["CS336_GEMM"] = gemm_mode_saved
    if tmode == "tune" and rank == 0:
        import torch.cuda.tunable as tunable

        log(f"TunableOp results are written to {tunable.get_filename()} at exit")
    rep = os.environ.get("CS336_GEMM_REPORT")
    if rep and rank == 0 and gemm_mode() == "best":  # per-problem candidate times of best mode
        from cs336_systems.ops.gemm import gemm_choices, gemm_timings

        ch = gemm_choices()
        with open(rep, "w") as fh:
            json.dump([{"key": str(k), "pick": ch.get(k), "ms": v} for k, v in gemm_timings().items()], fh, indent=1)
        with open(rep + ".lt.json", "w") as fh:  # autotuned hipBLASLt candidates (scripts/gemm_table.py pins)
            json.dump(sorted(torch.ops.cs336.lt_gemm_picks()), fh, indent=1)
    if rank == 0:
        emit_result(out, args.json_out)
    if dist.is_initialized():
        try:
            dist.barrier()
            dist.destroy_process_group()
        except Exception as e:  # noqa: BLE001 - a peer already left (sweep watchdog); the result line is out
            log(f"rank {rank}: teardown after the result line failed ({type(e).__name__}); exiting")
    return 0


if __name__ == "__main__":
    sys.exit(main())
