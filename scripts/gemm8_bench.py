"""gemm8 (each tile width) vs hipBLASLt (torch.mm default pick, and the autotuned cs336 lt_gemm) on a
model's NT projection GEMMs, random operands, interleaved rounds in one process.

    python scripts/gemm8_bench.py [--model xl|2p7b] [--tokens 49152] [--reps 20] [--rounds 3] [--json out.json]
"""

import argparse
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

# name, N, K, epi  (d_model D, d_ff F, vocab V)
def problems(D, F, V):
    return [
        ("qkv fwd", 3 * D, D, 0), ("o fwd", D, D, 0), ("w13 fwd+swiglu", 2 * F, D, 1), ("w2 fwd", D, F, 0),
        ("lm fwd", V, D, 0), ("w13 dX", D, 2 * F, 0), ("w2 dX+swiglu_bwd", F, D, 2), ("qkv dX", D, 3 * D, 0),
        ("o dX", D, D, 0), ("lm dX", D, V, 0),
    ]


MODELS = {"xl": (1600, 6400, 10000), "2p7b": (2560, 10240, 10000)}


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
    ap.add_argument("--model", default="xl", choices=sorted(MODELS))
    ap.add_argument("--tokens", type=int, default=49152)
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--json", default=None)
    ap.add_argument("--only", default=None)
    ap.add_argument("--gemm8-only", action="store_true", help="time gemm8 alone (variant A/B)")
    args = ap.parse_args()
    from cs336_systems import ops

    assert ops.load_ext(), ops.load_error()
    cs = torch.ops.cs336
    M = args.tokens
    rows = []
    for name, N, K, epi in problems(*MODELS[args.model]):
        if args.only and args.only not in name:
            continue
        g = torch.Generator(device="cuda").manual_seed(N + K)
        a = ((torch.rand(M, K, device="cuda", generator=g) * 2 - 1)).bfloat16()
        b = ((torch.rand(N, K, device="cuda", generator=g) * 2 - 1) * 0.05).bfloat16()
        half = N // 2 if epi == 1 else N
        c = torch.empty(M, N if epi != 2 else 2 * N, device="cuda", dtype=torch.bfloat16)
        h = torch.empty(M, half, device="cuda", dtype=torch.bfloat16) if epi == 1 else None
        y = ((torch.rand(M, 2 * N, device="cuda", generator=g) * 2 - 1) * 3).bfloat16() if epi == 2 else None
        cands = {}
        for fn in (5, 4):
            ok = (half % (32 * fn) == 0) if epi == 1 else (N % (64 * fn) == 0 or (epi == 0 and N % 8 == 0))
            if ok:
                cands[f"g8_fn{fn}"] = (lambda fn=fn: cs.gemm8(a, b, c, epi, fn, h, y, half))
        if not args.gemm8_only and epi == 0:
            cands["blas"] = lambda: torch.mm(a, b.t())
            cands["lt"] = lambda: cs.lt_gemm(a, b, False, True, torch.bfloat16)
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
        del a, b, c, h, y
        torch.cuda.empty_cache()
    if args.json:
        with open(args.json, "w") as f:
            json.dump(rows, f, indent=1)


if __name__ == "__main__":
    main()
