"""Time the model's GEMM shapes on MI355X across BLAS backends (hipBLASLt / rocBLAS) and the two
orientations of the weight-gradient GEMM, to build the per-shape selection table used by
cs336_systems/models/fused.py. Usage: python scripts/gemm_bench.py [M ...]"""

import json
import sys

import torch

sys.path.insert(0, ".")
from cs336_systems.utils.timing import do_bench  # noqa: E402


def main():
    Ms = [int(x) for x in sys.argv[1:]] or [8192, 12288, 16384]
    d, f, V = 1600, 6400, 10000
    shapes = {"qkv": (3 * d, d), "o": (d, d), "w13": (2 * f, d), "w2": (d, f), "lm": (V, d)}
    dev = "cuda"
    results = []
    for M in Ms:
        for name, (N, K) in shapes.items():
            x = torch.randn(M, K, device=dev, dtype=torch.bfloat16)
            w = torch.randn(N, K, device=dev, dtype=torch.bfloat16)
            dy = torch.randn(M, N, device=dev, dtype=torch.bfloat16)
            fl = 2.0 * M * N * K
            row = dict(M=M, name=name, N=N, K=K)
            for lib in ("cublaslt", "cublas"):  # = hipBLASLt, rocBLAS on ROCm
                torch.backends.cuda.preferred_blas_library(lib)
                tag = "lt" if lib == "cublaslt" else "rb"
                cases = {
                    "fwd": lambda: x @ w.t(),
                    "dx": lambda: dy @ w,
                    "dw_tn": lambda: torch.mm(dy.t(), x, out_dtype=torch.float32),
                    "dw_nt": lambda: torch.mm(x.t(), dy, out_dtype=torch.float32),
                    "dw_tn_bf16": lambda: dy.t() @ x,
                }
                for k, fn in cases.items():
                    try:
                        t = do_bench(fn, rep=30, warmup=5, flush_cache=False)[0]
                        row[f"{k}_{tag}"] = round(fl / (t * 1e-3) / 1e12)
                    except Exception as e:  # some combos unsupported by a backend
                        row[f"{k}_{tag}"] = None
            torch.backends.cuda.preferred_blas_library("cublaslt")
            results.append(row)
            print(json.dumps(row), flush=True)
    with open("gpurun_out/gemm_bench.json", "w") as fh:
        json.dump(results, fh, indent=1)


if __name__ == "__main__":
    main()
