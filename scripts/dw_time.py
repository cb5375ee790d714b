"""Time the XL step's weight-gradient GEMMs exactly as the step runs them (ops.gemm.mm_dw: gemm8w with
the committed split plan, fp32 out, slab reduction included) at the bench's 52,224 tokens, random
operands. One line of JSON per problem; run it once per library (CS336_LIB) for a same-box A/B:

    for r in 1 2; do for lib in base new; do CS336_LIB=... python scripts/dw_time.py --tag $lib; done; done
"""

from __future__ import annotations

import argparse
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

# name, N_out (dY columns), K_in (X columns)
PROBLEMS = [("w13 dW", 12800, 1600), ("w2 dW", 1600, 6400), ("qkv dW", 4800, 1600), ("o dW", 1600, 1600)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tokens", type=int, default=52224)
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--tag", default="")
    args = ap.parse_args()
    from cs336_systems import ops
    from cs336_systems.ops import gemm

    assert ops.load_ext(), ops.load_error()
    T = args.tokens
    for name, n, k in PROBLEMS:
        g = torch.Generator(device="cuda").manual_seed(n + k)
        dy = (torch.rand(T, n, device="cuda", generator=g) * 2 - 1).bfloat16()
        x = (torch.rand(T, k, device="cuda", generator=g) * 2 - 1).bfloat16()
        out = torch.empty(n, k, device="cuda", dtype=torch.float32)
        ts = []
        for _ in range(args.rounds):
            gemm.mm_dw(dy, x, out=out)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(args.reps):
                gemm.mm_dw(dy, x, out=out)
            e1.record()
            e1.synchronize()
            ts.append(e0.elapsed_time(e1) / args.reps)
        # numerics on a 4096-token slice against fp32
        ref = dy[:4096].float().t() @ x[:4096].float()
        got = gemm.mm_dw(dy[:4096], x[:4096])
        err = ((got - ref).abs().max() / ref.abs().max()).item()
        ms = statistics.median(ts)
        print(json.dumps({"tag": args.tag, "problem": name, "tokens": T, "ms": round(ms, 4),
                          "tflops": round(2.0 * T * n * k / ms / 1e9, 1), "plan": str(gemm.dw_launch_plan(dy, x)),
                          "max_rel_err_4096": err}), flush=True)
        del dy, x, out
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
