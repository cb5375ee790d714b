"""Autotuned hipBLASLt (``cs336::lt_gemm``, csrc/blas/lt_gemm.cpp) vs ``torch.mm`` on the XL
projection GEMMs, each in the operand layout :class:`FusedLinearFn` uses.

    python scripts/lt_gemm_sweep.py [--tokens 12288] [--json out.json]

Prints per GEMM: torch.mm time, tuned time, the heuristic's first pick as timed by the tuner, TFLOPS
and the max error of the tuned result against torch.mm (fp32 accumulate on both sides).
"""

from __future__ import annotations

import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from cs336_systems.ops._ext import ops  # noqa: E402


def timed(fn, reps=20):
    for _ in range(3):
        fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return 1000.0 * e0.elapsed_time(e1) / reps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tokens", type=int, default=12288)
    ap.add_argument("--d-model", type=int, default=1600)
    ap.add_argument("--d-ff", type=int, default=6400)
    ap.add_argument("--vocab", type=int, default=10000)
    ap.add_argument("--json", default=None)
    a = ap.parse_args()
    T, D, F, V = a.tokens, a.d_model, a.d_ff, a.vocab
    dev = "cuda"
    bf = torch.bfloat16
    projs = {"qkv": (3 * D, D), "o": (D, D), "w13": (2 * F, D), "w2": (D, F), "lm_head": (V, D)}
    rows = []
    for name, (n_out, n_in) in projs.items():
        x = torch.randn(T, n_in, device=dev, dtype=bf)
        dy = torch.randn(T, n_out, device=dev, dtype=bf)
        w = torch.randn(n_out, n_in, device=dev, dtype=bf) * 0.02
        wt = w.t().contiguous()
        xt = x.t().contiguous()
        cases = [
            # (label, torch fn, a, b, a_t, b_t, out dtype)
            ("fwd X·Wᵀ", lambda: torch.mm(x, w.t()), x, w, False, True, bf),
            ("dgrad dY·(Wᵀ)ᵀ", lambda: torch.mm(dy, wt.t()), dy, wt, False, True, bf),
            ("dgrad dY·W", lambda: torch.mm(dy, w), dy, w, False, False, bf),
            ("dW dYᵀ·X fp32", lambda: torch.mm(dy.t(), x, out_dtype=torch.float32), dy, x, True, False, torch.float32),
            ("dW dYᵀ·(Xᵀ)ᵀ fp32", lambda: torch.mm(dy.t(), xt.t(), out_dtype=torch.float32), dy, xt, True, True, torch.float32),
        ]
        for label, tfn, A, B, at, bt, odt in cases:
            M = A.shape[1] if at else A.shape[0]
            N = B.shape[0] if bt else B.shape[1]
            K = A.shape[0] if at else A.shape[1]
            flops = 2.0 * M * N * K
            t_ref = timed(tfn)
            out = torch.empty(M, N, device=dev, dtype=odt)
            ops().lt_gemm_out(A, B, at, bt, out)  # tunes on first call
            t_lt = timed(lambda: ops().lt_gemm_out(A, B, at, bt, out))
            t_ref = min(t_ref, timed(tfn))  # both orders: clocks drift between the two timings
            ref = tfn().float()
            err = (out.float() - ref).abs().max().item() / max(ref.abs().max().item(), 1e-6)
            row = dict(proj=name, gemm=label, M=M, N=N, K=K, torch_us=round(t_ref, 1), lt_us=round(t_lt, 1),
                       torch_tf=round(flops / t_ref / 1e6, 1), lt_tf=round(flops / t_lt / 1e6, 1),
                       speedup=round(t_ref / t_lt, 3), rel_err=err)
            rows.append(row)
            print(f"{name:8s} {label:20s} {M:6d}x{N:6d}x{K:6d}  torch {t_ref:8.1f} us {row['torch_tf']:7.1f} TF | "
                  f"lt {t_lt:8.1f} us {row['lt_tf']:7.1f} TF | x{row['speedup']:.3f}  err {err:.2e}", flush=True)
            assert err < 2e-2, (name, label, err)
    tab = ops().lt_gemm_table()
    print("tuned problems (m n k a_t b_t out n_cand best_idx best_ns first_ns):")
    for i in range(0, len(tab), 10):
        print("  ", tab[i:i + 10])
    if a.json:
        with open(a.json, "w") as fh:
            json.dump({"device": torch.cuda.get_device_name(0), "tokens": T, "rows": rows}, fh, indent=1)


if __name__ == "__main__":
    main()
