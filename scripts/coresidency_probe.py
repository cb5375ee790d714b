"""Co-residency probe: can an RCCL-shaped cohort (every channel block must be resident at once) get
all of its workgroups while hipBLASLt's stream-K GEMMs of the XL backward own the chip?

Main stream: the XL layer's backward GEMM sequence (default hipBLASLt picks, stream-K) at the bench's
24576 tokens per GPU, `--iters` times. Side stream: before each iteration, a one-workgroup sleep of a
varying length (so the cohort lands at different points of the GEMM sequence), then a cohort of
`--blocks` workgroups shaped like an RCCL gfx950 channel block (256 threads, 21,184 B LDS, 128
VGPRs) that waits, up to `--deadline-ms`, for all of its workgroups to arrive
(csrc/ops/occupy.hip ``cohort_kernel``). A stranded cohort is exactly the partially-resident RCCL
kernel of a cross-rank DDP deadlock; with the deadline it records a timeout instead of hanging.

Prints one JSON line: cohort launches, workgroups that timed out, the longest assembly wait, the
GEMM sequence's time with and without the cohort beside it, and the stream-K environment.

    python scripts/coresidency_probe.py [--blocks 32] [--iters 40]
    TENSILE_STREAMK_MAX_CUS=240 python scripts/coresidency_probe.py
"""

from __future__ import annotations

import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

# must precede the first hipBLASLt call (and, to be safe, the library's load): `--streamk-cap N`
# stands for the bench's multi-GPU setting (cs336_systems.parallel.comm.streamk_env)
if "--streamk-cap" in sys.argv:
    os.environ["TENSILE_STREAMK_MAX_CUS"] = sys.argv[sys.argv.index("--streamk-cap") + 1]

import torch  # noqa: E402

T, D, F = 24576, 1600, 6400  # bench.py XL: 48 x 512 tokens per GPU


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--blocks", type=int, default=32, help="cohort workgroups (RCCL channels)")
    ap.add_argument("--lds", type=int, default=21184)
    ap.add_argument("--iters", type=int, default=40)
    ap.add_argument("--deadline-ms", type=float, default=50.0)
    ap.add_argument("--streamk-cap", type=int, default=None)
    ap.add_argument("--race", action="store_true",
                    help="launch a cohort beside EVERY GEMM, released by an event recorded right before that GEMM, "
                         "so the cohort and the GEMM grid are dispatched at the same moment")
    args = ap.parse_args()

    from cs336_systems import ops

    assert ops.load_ext(), ops.load_error()
    cs = torch.ops.cs336
    g = torch.Generator(device="cuda").manual_seed(0)
    r = lambda *s: (torch.randn(*s, device="cuda", generator=g) * 0.05).to(torch.bfloat16)  # noqa: E731
    x, h, dy_o, dy_13, dy_qkv = r(T, D), r(T, F), r(T, D), r(T, 2 * F), r(T, 3 * D)
    w_2, w_13, w_o, w_qkv = r(D, F), r(2 * F, D), r(D, D), r(3 * D, D)

    gemms = [lambda: dy_o @ w_2, lambda: torch.mm(dy_o.t(), h, out_dtype=torch.float32), lambda: dy_13 @ w_13,
             lambda: torch.mm(dy_13.t(), x, out_dtype=torch.float32), lambda: dy_o @ w_o,
             lambda: torch.mm(dy_o.t(), x, out_dtype=torch.float32), lambda: dy_qkv @ w_qkv,
             lambda: torch.mm(dy_qkv.t(), x, out_dtype=torch.float32)]

    def seq(before=None):
        out = []
        for g in gemms:
            if before is not None:
                before()
            out.append(g())
        return out

    ref = seq()
    torch.cuda.synchronize()

    def timed(n, with_cohort):
        state = torch.zeros(3, dtype=torch.int32, device="cuda")
        sleeper = torch.zeros(1, dtype=torch.int32, device="cuda")
        main = torch.cuda.current_stream()
        side = torch.cuda.Stream()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        def racer():
            side.wait_stream(main)  # released when the previous GEMM ends, like the next one
            with torch.cuda.stream(side):
                cs.cohort(args.blocks, args.lds, args.deadline_ms, state)

        for i in range(n):
            if with_cohort and not args.race:
                side.wait_stream(main)
                with torch.cuda.stream(side):
                    cs.occupy(1, 4, (i * 0.37) % 3.0, sleeper)  # land at varying points of seq()
                    cs.cohort(args.blocks, args.lds, args.deadline_ms, state)
            out = seq(racer if with_cohort and args.race else None)
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / n
        return dt, state.tolist(), out

    base_s, _, _ = timed(args.iters, False)
    co_s, st, out = timed(args.iters, True)
    ok = all(torch.equal(a, b) for a, b in zip(out, ref))
    res = {
        "mode": "race" if args.race else "staggered", "blocks": args.blocks, "lds": args.lds, "iters": args.iters, "deadline_ms": args.deadline_ms,
        "cohort_timeouts_wg": st[1], "max_assembly_wait_ms": round(st[2] / 1e5, 3),
        "gemm_seq_ms": round(base_s * 1e3, 3), "gemm_seq_ms_with_cohort": round(co_s * 1e3, 3),
        "results_bitwise_equal": ok,
        "env": {k: v for k, v in os.environ.items() if k.startswith(("TENSILE_", "NCCL_", "HIPBLASLT"))},
    }
    print(json.dumps(res), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
