"""gemm8 vs hipBLASLt (torch.mm default pick, and the autotuned cs336 lt_gemm) on the XL step's NT
projection GEMMs at 24576 tokens, random operands, interleaved rounds in one process.

    python scripts/gemm8_bench.py [--reps 20] [--rounds 3] [--json out.json]
"""

import argparse
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

M = 24576
# name, N, K, epi
PROBLEMS = [
    ("qkv fwd", 4800, 1600, 0), ("o fwd", 1600, 1600, 0), ("w13 fwd", 12800, 1600, 0), ("w13 fwd+swiglu", 12800, 1600, 1),
    ("w2 fwd", 1600, 6400, 0), ("w13 dX", 1600, 12800, 0), ("w2 dX", 6400, 1600, 0), ("w2 dX+swiglu_bwd", 6400, 1600, 2),
    ("qkv dX", 1600, 4800, 0), ("o dX", 1600, 1600, 0),
]


def timeit(fn, reps):
    fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    e1.synchronize()
    return e0.elapsed_time(e1) / reps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--json", default=None)
    ap.add_argument("--only", default=None)
    ap.add_argument("--gemm8-only", action="store_true", help="time gemm8 alone (variant A/B)")
    args = ap.parse_args()
    from cs336_systems import ops

    assert ops.load_ext(), ops.load_error()
    cs = torch.ops.cs336
    rows = []
    for name, N, K, epi in PROBLEMS:
        if args.only and args.only not in name:
            continue
        g = torch.Generator(device="cuda").manual_seed(N + K)
        a = ((torch.rand(M, K, device="cuda", generator=g) * 2 - 1)).bfloat16()
        b = ((torch.rand(N, K, device="cuda", generator=g) * 2 - 1) * 0.05).bfloat16()
        half = N // 2 if epi == 1 else N
        c = torch.empty(M, N if epi != 2 else 2 * N, device="cuda", dtype=torch.bfloat16)
        h = torch.empty(M, half, device="cuda", dtype=torch.bfloat16) if epi == 1 else None
        y = ((torch.rand(M, 2 * N, device="cuda", generator=g) * 2 - 1) * 3).bfloat16() if epi == 2 else None
        cands = {
            "gemm8": lambda: cs.gemm8(a, b, c, epi, 0, h, y, half),
            "blas": lambda: torch.mm(a, b.t()),
            "lt": lambda: cs.lt_gemm(a, b, False, True, torch.bfloat16),
        }
        if args.gemm8_only:
            cands = {"gemm8": cands["gemm8"]}
        elif epi == 1:  # unfused reference pipeline: GEMM + SwiGLU kernel
            cands["blas+swiglu"] = lambda: cs.swiglu_fused_fwd(torch.mm(a, b.t()))
        if epi == 2 and not args.gemm8_only:
            cands["blas+swiglu_bwd"] = lambda: cs.swiglu_fused_bwd(torch.mm(a, b.t()), y)
        times = {k: [] for k in cands}
        for _ in range(args.rounds):
            for k, fn in cands.items():
                times[k].append(timeit(fn, args.reps))
        flop = 2.0 * M * N * K
        row = {"problem": name, "M": M, "N": N, "K": K, "epi": epi}
        for k, v in times.items():
            ms = statistics.median(v)
            row[k + "_ms"] = round(ms, 4)
            row[k + "_tflops"] = round(flop / ms / 1e9, 1)
        rows.append(row)
        print(json.dumps(row), flush=True)
    if args.json:
        with open(args.json, "w") as f:
            json.dump(rows, f, indent=1)


if __name__ == "__main__":
    main()
