"""gemm8w vs the current weight-gradient GEMMs (hipBLASLt default, autotuned lt, torch split-K) on the
XL step's four dW problems at 24576 tokens, random operands, interleaved rounds in one process.
Each problem tries gemm8w in both roles (plain / transposed store) and several split-K counts; split-K
times include the slab reduction.

    python scripts/gemm8w_bench.py [--json out.json]
"""

import argparse
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
T = 24576
PROBLEMS = [("w13 dW", 12800, 1600), ("w2 dW", 1600, 6400), ("qkv dW", 4800, 1600), ("o dW", 1600, 1600), ("lm dW", 10000, 1600)]


def timeit(fn, reps=10):
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
    ap.add_argument("--json", default=None)
    ap.add_argument("--tokens", type=int, default=24576)
    ap.add_argument("--rounds", type=int, default=3)
    args = ap.parse_args()
    global T
    T = args.tokens
    from cs336_systems import ops

    assert ops.load_ext(), ops.load_error()
    cs = torch.ops.cs336
    rows = []
    for name, n_out, k_in in PROBLEMS:
        g = torch.Generator(device="cuda").manual_seed(n_out + k_in)
        dy = (torch.rand(T, n_out, device="cuda", generator=g) * 2 - 1).bfloat16()
        x = (torch.rand(T, k_in, device="cuda", generator=g) * 2 - 1).bfloat16()
        out = torch.empty(n_out, k_in, device="cuda")
        cands = {"blas": lambda: torch.mm(dy.t(), x, out_dtype=torch.float32, out=out),
                 "lt": lambda: cs.lt_gemm_out(dy, x, True, False, out)}
        for trans in (False, True):
            a, b = (x, dy) if trans else (dy, x)  # trans: compute dWᵀ tiles, store transposed
            M, N = a.shape[1], b.shape[1]
            if not (N % 320 == 0 or N % 256 == 0):
                continue
            for sk in (1, 2, 3, 4, 5, 6, 7, 8):
                if (T // 64) < sk:
                    continue
                tag = f"g8w{'T' if trans else ''}_s{sk}"
                if sk == 1:
                    cands[tag] = lambda a=a, b=b, trans=trans: cs.gemm8w(a, b, out, 1, trans, False, 0)
                else:
                    slabs = torch.empty(sk, n_out, k_in, device="cuda")

                    def run(a=a, b=b, trans=trans, sk=sk, slabs=slabs):
                        cs.gemm8w(a, b, slabs, sk, trans, False, 0)
                        torch.sum(slabs, dim=0, out=out)

                    cands[tag] = run
        ref = torch.mm(dy.t(), x, out_dtype=torch.float32)
        times = {k: [] for k in cands}
        errs = {}
        for _ in range(args.rounds):
            for k, fn in cands.items():
                times[k].append(timeit(fn))
                if k not in errs:
                    errs[k] = float((out - ref).norm() / ref.norm())
        flop = 2.0 * T * n_out * k_in
        med = {k: statistics.median(v) for k, v in times.items()}
        best_g8w = min((k for k in med if k.startswith("g8w")), key=med.get)
        row = {"problem": name, "N_out": n_out, "K_in": k_in, "ms": {k: round(v, 4) for k, v in med.items()},
               "best_g8w": best_g8w, "best_g8w_tflops": round(flop / med[best_g8w] / 1e9, 1),
               "blas_tflops": round(flop / med["blas"] / 1e9, 1), "lt_tflops": round(flop / med["lt"] / 1e9, 1),
               "max_rel_err": max(errs.values())}
        rows.append(row)
        print(json.dumps(row), flush=True)
        del dy, x, out, cands
        torch.cuda.empty_cache()
    if args.json:
        with open(args.json, "w") as f:
            json.dump(rows, f, indent=1)


if __name__ == "__main__":
    main()
