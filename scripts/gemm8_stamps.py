"""Where a gemm8 tile's time goes, from in-kernel stamps (diagnostic build, -DCS336_G8_STAMP).

    CS336_BUILD_VARIANT="stamp -DCS336_G8_STAMP=1" python -m cs336_systems._native.build
    CS336_LIB=cs336_systems/_native/variants/stamp/libcs336_hip.so python scripts/gemm8_stamps.py [--tokens 52224]

For each XL projection problem (random operands, one warm launch, then a stamped one) every
workgroup records s_memtime at its start, after the prologue (k-tiles 0/1 landed, first barrier),
after the main loop and after its epilogue's stores retired (an added vmcnt(0): the stamped build
waits for them, the shipped one does not), plus its CU (HW_ID, XCC_ID). Reported per problem, in
shader cycles (median over workgroups): prologue, main loop, epilogue, and per CU the gap between
one workgroup's end and the next one's start on that CU (dispatch + launch overhead), plus the
clock (memtime ticks per memrealtime tick x 100 MHz) and each phase's share of the busy span.
"""

from __future__ import annotations

import argparse
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

# name, N, K, epi (M = tokens), per model
PROBLEMS = {
    "xl": [
        ("o fwd", 1600, 1600, 0),
        ("qkv fwd (plain)", 4800, 1600, 0),
        ("w13 fwd+swiglu", 12800, 1600, 1),
        ("w2 dX+swiglu_bwd", 6400, 1600, 2),
        ("w2 fwd", 1600, 6400, 0),
        ("w13 dX", 1600, 12800, 0),
    ],
    "2p7b": [
        ("o fwd", 2560, 2560, 0),
        ("qkv fwd (plain)", 7680, 2560, 0),
        ("w13 fwd+swiglu", 20480, 2560, 1),
        ("w2 dX+swiglu_bwd", 10240, 2560, 2),
        ("w2 fwd", 2560, 10240, 0),
        ("qkv dX", 2560, 7680, 0),
    ],
}


def analyse(st: torch.Tensor) -> dict:
    s = st.cpu().tolist()
    pro = [r[1] - r[0] for r in s]
    main = [r[2] - r[1] for r in s]
    epi = [r[3] - r[2] for r in s]
    tot = [r[3] - r[0] for r in s]
    clk = [(r[3] - r[0]) / max(1, r[5] - r[4]) * 0.1 for r in s]  # GHz
    # per CU: consecutive workgroups (by start) -> gap = next start - previous end
    by_cu: dict = {}
    for r in s:
        hw, xcc = int(r[6]), int(r[7])
        cu = (xcc & 0xF, (hw >> 13) & 0x7, (hw >> 12) & 0x1, (hw >> 8) & 0xF)  # xcc, se, sh, cu
        by_cu.setdefault(cu, []).append((r[0], r[3]))
    gaps = []
    for v in by_cu.values():
        v.sort()
        gaps += [b[0] - a[1] for a, b in zip(v, v[1:])]
    t_first, t_last = min(r[0] for r in s), max(r[3] for r in s)
    med = statistics.median
    return {
        "workgroups": len(s), "cus": len(by_cu), "clock_ghz": round(med(clk), 3),
        "prologue_cyc": round(med(pro)), "main_cyc": round(med(main)), "epilogue_cyc": round(med(epi)),
        "tile_cyc": round(med(tot)), "gap_cyc_median": round(med(gaps)) if gaps else None,
        "gap_cyc_p90": round(sorted(gaps)[int(0.9 * len(gaps))]) if gaps else None,
        "span_cyc": t_last - t_first,
        "share": {k: round(med(x) / med(tot), 3) for k, x in (("prologue", pro), ("main", main), ("epilogue", epi))},
    }


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tokens", type=int, default=52224)
    ap.add_argument("--model", choices=sorted(PROBLEMS), default="xl")
    ap.add_argument("--json", default=None)
    args = ap.parse_args()
    from cs336_systems import ops

    assert ops.load_ext(), ops.load_error()
    cs = torch.ops.cs336
    M = args.tokens
    rows = []
    for name, N, K, epi in PROBLEMS[args.model]:
        g = torch.Generator(device="cuda").manual_seed(N + K)
        a = (torch.rand(M, K, device="cuda", generator=g) * 2 - 1).bfloat16()
        half = N // 2 if epi == 1 else N
        b = ((torch.rand(N, K, device="cuda", generator=g) * 2 - 1) * 0.05).bfloat16()
        c = torch.empty(M, N if epi != 2 else 2 * N, device="cuda", dtype=torch.bfloat16)
        h = torch.empty(M, half, device="cuda", dtype=torch.bfloat16) if epi == 1 else None
        y = ((torch.rand(M, 2 * N, device="cuda", generator=g) * 2 - 1) * 3).bfloat16() if epi == 2 else None
        blocks = (M // 256) * (N // 320)
        st = torch.zeros(blocks, 8, dtype=torch.int64, device="cuda")
        for _ in range(3):
            cs.gemm8(a, b, c, epi, 5, h, y, half)
        torch.cuda.synchronize()
        if not cs.gemm8_stamps(st):
            raise SystemExit("this build writes no stamps: build the CS336_G8_STAMP variant and load it with CS336_LIB")
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        cs.gemm8(a, b, c, epi, 5, h, y, half)
        e1.record()
        torch.cuda.synchronize()
        cs.gemm8_stamps(None)
        row = {"model": args.model, "problem": name, "M": M, "N": N, "K": K, "epi": epi, "ms": round(e0.elapsed_time(e1), 4), **analyse(st)}
        rows.append(row)
        print(json.dumps(row), flush=True)
        del a, b, c, h, y, st
        torch.cuda.empty_cache()
    if args.json:
        with open(args.json, "w") as f:
            json.dump(rows, f, indent=1)


if __name__ == "__main__":
    main()
