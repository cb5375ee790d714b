"""Kernel launch sequence of one layer of the last full step in a rocprofv3 kernel trace (short
names, duration, stream): shows which small kernels (fills, copies, casts) a layer's forward and
backward launch. usage: python scripts/step_sequence.py <kernel_trace.csv> [--layer 10]"""

import argparse
import csv
import re


def short(n):
    if n.startswith("Cijk") or n.startswith("Custom_Cijk"):
        m = re.search(r"MT\d+x\d+x\d+", n)
        return "GEMM " + (m.group(0) if m else "")
    m = re.search(r"(\w+_kernel)\b", n)
    base = m.group(1) if m else n.split("(")[0][:60]
    f = re.search(r"(FillFunctor<[\w:]+>|direct_copy|CUDAFunctor\w*|MulFunctor|copyBuffer|fillBuffer\w*)", n)
    return base + (" " + f.group(1) if f else "")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--layer", type=int, default=10)
    a = ap.parse_args()
    rows = list(csv.DictReader(open(a.trace)))
    iv = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"], r.get("Stream_Id", "")) for r in rows)
    starts = [s for s, _, n, _ in iv if "vectorized_gather_kernel" in n]
    lo, hi = starts[-2], starts[-1]
    step = [x for x in iv if lo <= x[0] < hi]
    fwd_fa = [i for i, x in enumerate(step) if "fa_fwd" in x[2]]
    # one FA backward anchor per layer: the two-kernel form's dQ kernel, the fused kernel, the kp prep
    # launch, or the hs main kernel (its prep launch, when CS336_FA_HS_DELTA=0, then ends the listing
    # of the layer before)
    anchors = ("fa_bwd_dq", "fa_bwd_fused", "fa_bwd_kp_prep", "fa_bwd_hs_kernel")
    bwd_fa = [i for i, x in enumerate(step) if any(a in x[2] for a in anchors)]
    L = a.layer
    print(f"== forward, layer {L}")
    for x in step[fwd_fa[L]:fwd_fa[L + 1]]:
        print(f"{(x[1] - x[0]) / 1e3:9.1f} us  s{x[3]}  {short(x[2])}")
    print(f"== backward, between FA bwd of layer {len(bwd_fa) - 1 - L} and the next")
    for x in step[bwd_fa[L]:bwd_fa[L + 1]]:
        print(f"{(x[1] - x[0]) / 1e3:9.1f} us  s{x[3]}  {short(x[2])}")
    print("== after the last layer's backward (optimizer etc.)")
    for x in step[bwd_fa[-1]:]:
        print(f"{(x[1] - x[0]) / 1e3:9.1f} us  s{x[3]}  {short(x[2])}")


if __name__ == "__main__":
    main()
