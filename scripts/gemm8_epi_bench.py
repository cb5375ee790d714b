"""Time gemm8 (csrc/gemm/gemm8.hip) on the XL step's NT projection problems (epilogues 0-2) at 49152
tokens, random operands, interleaved rounds in one process; with --check the repeated calls must
agree bitwise. Used per variant build by scripts/g8_variants.sh (CS336_LIB).

    python scripts/gemm8_epi_bench.py [--rounds 3] [--reps 10] [--only swiglu]
"""

import argparse
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

# name, M, N, K, epi
PROBLEMS = [
    ("w13 fwd+swiglu", 49152, 12800, 1600, 1),
    ("w2 dX+swiglu_bwd", 49152, 6400, 1600, 2),
    ("qkv fwd", 49152, 4800, 1600, 0),
    ("w2 fwd", 49152, 1600, 6400, 0),
    ("w13 dX", 49152, 1600, 12800, 0),
    ("o fwd", 49152, 1600, 1600, 0),
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
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--only", default=None)
    ap.add_argument("--json", default=None)
    ap.add_argument("--no-check", action="store_true", help="skip the bitwise repeat check (ablation builds)")
    args = ap.parse_args()
    from cs336_systems import ops

    assert ops.load_ext(), ops.load_error()
    cs = torch.ops.cs336
    rows = []
    for name, M, N, K, epi in PROBLEMS:
        if args.only and args.only not in name:
            continue
        g = torch.Generator(device="cuda").manual_seed(N + K)
        a = (torch.rand(M, K, device="cuda", generator=g) * 2 - 1).bfloat16()
        b = ((torch.rand(N, K, device="cuda", generator=g) * 2 - 1) * 0.05).bfloat16()
        half = N // 2 if epi == 1 else N
        c = torch.empty(M, N if epi != 2 else 2 * N, device="cuda", dtype=torch.bfloat16)
        h = torch.empty(M, half, device="cuda", dtype=torch.bfloat16) if epi == 1 else None
        y = ((torch.rand(M, 2 * N, device="cuda", generator=g) * 2 - 1) * 3).bfloat16() if epi == 2 else None
        ref = None
        times = []
        for _ in range(args.rounds):
            times.append(timeit(lambda: cs.gemm8(a, b, c, epi, 0, h, y, half), args.reps))
            if args.no_check:
                pass
            elif ref is None:
                ref = c.clone()
            else:  # repeated launches are deterministic
                assert torch.equal(ref, c), f"{name}: result changed between calls"
        flop = 2.0 * M * N * K
        ms = statistics.median(times)
        row = {"problem": name, "M": M, "N": N, "K": K, "epi": epi,
               "ms": round(ms, 4), "min_ms": round(min(times), 4), "tflops": round(flop / ms / 1e9, 1)}
        rows.append(row)
        print(json.dumps(row), flush=True)
        del a, b, c, h, y, ref
        torch.cuda.empty_cache()
    if args.json:
        with open(args.json, "w") as f:
            json.dump(rows, f, indent=1)


if __name__ == "__main__":
    main()
