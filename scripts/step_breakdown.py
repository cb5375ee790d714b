"""Per-phase, per-stream kernel time of the last full training step in a rocprofv3 kernel trace
(steps delimited by the embedding gather kernel; forward ends at the cross-entropy kernel).

    python scripts/step_breakdown.py <run>_kernel_trace.csv [--top 30]
"""

import argparse
import csv
import re
from collections import defaultdict


def short(n):
    if n.startswith("Cijk") or n.startswith("Custom"):
        m = re.search(r"MT(\d+x\d+x\d+)", n)
        return "GEMM " + n[:14] + " " + (m.group(1) if m else "")
    return n[:70]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--top", type=int, default=30)
    a = ap.parse_args()
    rows = list(csv.DictReader(open(a.trace)))
    iv = sorted(
        (int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"], r["Stream_Id"], int(r["Grid_Size_X"]) // max(1, int(r["Workgroup_Size_X"])))
        for r in rows
    )
    starts = [x[0] for x in iv if "vectorized_gather_kernel" in x[2]]
    lo, hi = starts[-2], starts[-1]
    w = [x for x in iv if lo <= x[0] < hi]
    xf = [x for x in w if "xent_fwd" in x[2]][0][0]
    print(f"step {(hi - lo) / 1e6:.2f} ms")
    for name, (p0, p1) in {"forward": (lo, xf), "backward+optimizer": (xf, hi)}.items():
        agg = defaultdict(lambda: [0, 0.0])
        for s, e, n, q, g in w:
            if p0 <= s < p1:
                k = (q, short(n), g)
                agg[k][0] += 1
                agg[k][1] += (e - s) / 1e3
        print(f"=== {name}: {(p1 - p0) / 1e6:.2f} ms")
        for k, (c, t) in sorted(agg.items(), key=lambda x: -x[1][1])[: a.top]:
            print(f"  stream {k[0]} {t / 1e3:8.2f} ms  n={c:4d}  avg {t / c:8.1f} us  wgs {k[2]:6d}  {k[1]}")


if __name__ == "__main__":
    main()
