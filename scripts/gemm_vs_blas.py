"""Time the cs336 MFMA GEMM against hipBLASLt (torch.mm) on the model's projection GEMMs in the
three training orientations. Usage: python scripts/gemm_vs_blas.py [--tokens 12288] [--d 1600 --ff 6400]
Prints one JSON row per (shape, orientation) with TFLOPS of both and the tile plan."""

import argparse
import json
import sys

import torch

sys.path.insert(0, ".")
from cs336_systems.ops._ext import ops as _hip  # noqa: E402
from cs336_systems.utils.timing import do_bench  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tokens", type=int, default=12288)
    ap.add_argument("--d", type=int, default=1600)
    ap.add_argument("--ff", type=int, default=6400)
    ap.add_argument("--tiles", action="store_true", help="also time every explicit tile")
    ap.add_argument("--json", default=None)
    args = ap.parse_args()
    h = _hip()
    T, d, f = args.tokens, args.d, args.ff
    shapes = {"qkv": (3 * d, d), "o": (d, d), "w13": (2 * f, d), "w2": (d, f)}
    rows = []
    for name, (N, K) in shapes.items():
        x = torch.randn(T, K, device="cuda").bfloat16()
        w = torch.randn(N, K, device="cuda").bfloat16()
        dy = torch.randn(T, N, device="cuda").bfloat16()
        fl = 2.0 * T * N * K
        dyT, xT = dy.t().contiguous(), x.t().contiguous()  # token-contiguous copies
        wT = w.t().contiguous()
        cases = {
            # name: (torch fn, a, b, trans_a, trans_b, out dtype)
            "fwd": (lambda: x @ w.t(), x, w, False, True, torch.bfloat16),
            "dx": (lambda: dy @ w, dy, w, False, False, torch.bfloat16),
            # input gradient from a transposed weight copy Wᵀ (K_in, N_out): both operands K-major
            "dx_wt": (lambda: dy @ wT.t(), dy, wT, False, True, torch.bfloat16),
            "dw": (lambda: torch.mm(dy.t(), x, out_dtype=torch.float32), dy, x, True, False, torch.float32),
            # the same weight gradient from token-contiguous (K-major) operands
            "dw_kk": (lambda: torch.mm(dyT, xT.t(), out_dtype=torch.float32), dyT, xT, False, True, torch.float32),
            # mixed: only X token-contiguous (saved transposed from the forward) / only dY
            "dw_xt": (lambda: torch.mm(dy.t(), xT.t(), out_dtype=torch.float32), dy, xT, True, True, torch.float32),
            "dw_dyt": (lambda: torch.mm(dyT, x, out_dtype=torch.float32), dyT, x, False, False, torch.float32),
            # input gradient from a transposed dYᵀ (N_out, tokens): A operand M-contiguous
            "dx_dyt": (lambda: dyT.t() @ w, dyT, w, True, False, torch.bfloat16),
            "dx_dyt_wt": (lambda: dyT.t() @ wT.t(), dyT, wT, True, True, torch.bfloat16),
            # the model's layout: dY and X both token-major (A and B MN-major)
            "dw": (lambda: torch.mm(dy.t(), x, out_dtype=torch.float32), dy, x, True, False, torch.float32),
        }
        for case, (tfn, a, b, ta, tb, odt) in cases.items():
            M_, N_ = (a.shape[1] if ta else a.shape[0]), (b.shape[0] if tb else b.shape[1])
            K_ = a.shape[0] if ta else a.shape[1]
            row = dict(shape=name, case=case, M=M_, N=N_, K=K_, plan=list(h.gemm_plan(M_, N_, K_, odt == torch.float32)))
            t_blas = do_bench(tfn, rep=40, warmup=5, flush_cache=False)[0]
            row["blas_tflops"] = round(fl / t_blas / 1e9)
            if h.gemm_ok(a, b, ta, tb):
                ref = tfn().float()
                got = h.gemm(a, b, ta, tb, odt, 0, 0, 0).float()
                row["max_rel_err"] = float((got - ref).abs().max() / ref.abs().max())
                t = do_bench(lambda: h.gemm(a, b, ta, tb, odt, 0, 0, 0), rep=40, warmup=5, flush_cache=False)[0]
                row["cs336_tflops"] = round(fl / t / 1e9)
                if args.tiles:
                    for bm, bn in ((256, 160), (160, 256), (192, 160), (160, 160)):
                        if M_ % bm == 0 and N_ % bn == 0:
                            for s in (1, 2, 4) if odt == torch.float32 else (1,):
                                t = do_bench(lambda: h.gemm(a, b, ta, tb, odt, bm, bn, s), rep=20, warmup=3, flush_cache=False)[0]
                                row[f"t{bm}x{bn}s{s}"] = round(fl / t / 1e9)
            rows.append(row)
            print(json.dumps(row), flush=True)
    if args.json:
        with open(args.json, "w") as fh:
            json.dump(rows, fh, indent=1)


if __name__ == "__main__":
    main()
