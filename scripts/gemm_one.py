"""Run one model GEMM (shape x orientation) a few times with either the cs336 kernel or hipBLASLt,
for rocprofv3 counter collection. Usage: python scripts/gemm_one.py w13 dx cs336|blas [reps]"""

import sys

import torch

sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__))))
from cs336_systems.ops._ext import ops as _hip  # noqa: E402


def main():
    shape, case, impl = sys.argv[1], sys.argv[2], sys.argv[3]
    reps = int(sys.argv[4]) if len(sys.argv) > 4 else 10
    T, d, f = 12288, 1600, 6400
    N, K = {"qkv": (3 * d, d), "o": (d, d), "w13": (2 * f, d), "w2": (d, f)}[shape]
    x = torch.randn(T, K, device="cuda").bfloat16()
    w = torch.randn(N, K, device="cuda").bfloat16()
    dy = torch.randn(T, N, device="cuda").bfloat16()
    h = _hip()
    if case == "fwd":
        a, b, ta, tb, odt, tfn = x, w, False, True, torch.bfloat16, lambda: x @ w.t()
    elif case == "dx":
        a, b, ta, tb, odt, tfn = dy, w, False, False, torch.bfloat16, lambda: dy @ w
    else:
        a, b, ta, tb, odt, tfn = dy, x, True, False, torch.float32, lambda: torch.mm(dy.t(), x, out_dtype=torch.float32)
    fn = (lambda: h.gemm(a, b, ta, tb, odt, 0, 0, 0)) if impl == "cs336" else tfn
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()


if __name__ == "__main__":
    main()
