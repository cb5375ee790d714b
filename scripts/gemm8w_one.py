"""Run one gemm8w problem a few times (for rocprofv3 --pmc passes): dW = dYᵀX of the XL W1|W3
(default), or the NT gemm8 W1|W3 input gradient (--nt) for comparison.

    python scripts/gemm8w_one.py [--nt] [--reps 5] [--n-out 12800 --k-in 1600 --splits 1 --trans 0]
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--nt", action="store_true")
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--tokens", type=int, default=24576)
    ap.add_argument("--n-out", type=int, default=12800)
    ap.add_argument("--k-in", type=int, default=1600)
    ap.add_argument("--splits", type=int, default=1)
    ap.add_argument("--trans", type=int, default=0)
    a = ap.parse_args()
    from cs336_systems import ops

    assert ops.load_ext(), ops.load_error()
    cs = torch.ops.cs336
    T = a.tokens
    g = torch.Generator(device="cuda").manual_seed(0)
    if a.nt:
        x = (torch.rand(T, a.n_out, device="cuda", generator=g) * 2 - 1).bfloat16()
        w = (torch.rand(a.k_in, a.n_out, device="cuda", generator=g) * 2 - 1).bfloat16()
        c = torch.empty(T, a.k_in, device="cuda", dtype=torch.bfloat16)
        fn = lambda: cs.gemm8(x, w, c, 0, 0, None, None, 0)  # noqa: E731
    else:
        dy = (torch.rand(T, a.n_out, device="cuda", generator=g) * 2 - 1).bfloat16()
        x = (torch.rand(T, a.k_in, device="cuda", generator=g) * 2 - 1).bfloat16()
        A, B = (x, dy) if a.trans else (dy, x)
        out = torch.empty((a.splits, a.n_out, a.k_in) if a.splits > 1 else (a.n_out, a.k_in), device="cuda")
        fn = lambda: cs.gemm8w(A, B, out, a.splits, bool(a.trans), False, 0)  # noqa: E731
    for _ in range(a.reps):
        fn()
    torch.cuda.synchronize()
    print("done", flush=True)


if __name__ == "__main__":
    main()
