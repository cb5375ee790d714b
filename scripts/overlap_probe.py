"""Two independent kernels of the XL backward, alone and on two HIP streams at once.

The FFN backward's W2 input-gradient GEMM (gemm8 EPI 2) ends in a memory-bound SwiGLU epilogue
(reads a, b, writes da, db: 8 B per output element) that runs while the matrix cores idle; the W2
weight gradient (gemm8w) is independent of it and compute-bound. Likewise the FA2 backward (latency
bound at N = 512) and the output projection's weight gradient. This measures what running each pair
concurrently buys over running it back to back:

    python scripts/overlap_probe.py --json gpurun_out/overlap.json
"""

import argparse
import os
import sys
import json

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))

from cs336_systems.ops import gemm
from cs336_systems.ops._ext import ops as _hip


def timeit(fn, reps=20, warm=3):
    for _ in range(warm):
        fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        fn()
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1))
    ts.sort()
    return ts[len(ts) // 2]


def pair(name, fa, fb, side):
    main = torch.cuda.current_stream()

    def both_serial():
        fa()
        fb()

    def both_conc():
        side.wait_stream(main)
        with torch.cuda.stream(side):
            fb()
        fa()
        main.wait_stream(side)

    def both_conc_rev():
        side.wait_stream(main)
        with torch.cuda.stream(side):
            fa()
        fb()
        main.wait_stream(side)

    r = dict(pair=name, a_ms=timeit(fa), b_ms=timeit(fb), serial_ms=timeit(both_serial),
             concurrent_ms=timeit(both_conc), concurrent_rev_ms=timeit(both_conc_rev))
    r["gain_ms"] = r["serial_ms"] - min(r["concurrent_ms"], r["concurrent_rev_ms"])
    print(json.dumps(r), flush=True)
    return r


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tokens", type=int, default=48 * 512)
    ap.add_argument("--json", default=None)
    a = ap.parse_args()
    T, d, dff, H, N = a.tokens, 1600, 6400, 25, 512
    B = T // N
    dev = "cuda"
    bf = torch.bfloat16
    torch.manual_seed(0)
    r = lambda *s: torch.randn(*s, device=dev, dtype=bf) * 0.05  # noqa: E731
    side = torch.cuda.Stream()
    rows = []

    # FFN: W2 input gradient with the SwiGLU epilogue  ||  W2 weight gradient
    dy, w2t, y, h = r(T, d), r(dff, d), r(T, 2 * dff), r(T, dff)
    dw2 = torch.empty(d, dff, device=dev, dtype=torch.float32)
    assert gemm.gemm8_ok(dy, w2t, 2, dff)
    rows.append(pair("w2_dx_epi2 || w2_dw", lambda: gemm.gemm8_swiglu_bwd(dy, w2t, y),
                     lambda: gemm.mm_dw(dy, h, out=dw2), side))

    # FFN: W1|W3 input gradient  ||  W1|W3 weight gradient
    dab, w13t, x = r(T, 2 * dff), r(d, 2 * dff), r(T, d)
    dw13 = torch.empty(2 * dff, d, device=dev, dtype=torch.float32)
    rows.append(pair("w13_dx || w13_dw", lambda: gemm.mm_nt(dab, w13t), lambda: gemm.mm_dw(dab, x, out=dw13), side))

    # attention: FA2 backward (B, H, N, 64) causal  ||  output-projection weight gradient
    q, k, v, o, do = (r(B, N, H, 64).transpose(1, 2) for _ in range(5))
    lse = torch.randn(B, H, N, device=dev, dtype=torch.float32) + 5.0
    dq, dk, dv = (torch.empty(B, N, H, 64, device=dev, dtype=bf).transpose(1, 2) for _ in range(3))
    hip = _hip()
    o2, x2 = r(T, d), r(T, d)
    dwo = torch.empty(d, d, device=dev, dtype=torch.float32)
    rows.append(pair("fa_bwd || o_dw", lambda: hip.fa_bwd_into(do, q, k, v, o, lse, True, 0.125, dq, dk, dv),
                     lambda: gemm.mm_dw(o2, x2, out=dwo), side))
    # attention: FA2 backward || QKV weight gradient of the next (earlier) layer is NOT independent;
    # the o-projection input gradient feeds the FA2 backward. FA2 forward || nothing independent.
    if a.json:
        with open(a.json, "w") as f:
            json.dump(rows, f, indent=1)


if __name__ == "__main__":
    main()
