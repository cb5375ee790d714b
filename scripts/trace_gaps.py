"""GPU occupancy of a rocprofv3 kernel trace: union of kernel intervals (all streams) vs wall span,
plus the largest idle gaps.

    python scripts/trace_gaps.py <run>_kernel_trace.csv [--last-frac 0.5] [--top 15]

Only the last ``--last-frac`` of the trace (by time) is analysed, so warmup/init is excluded.
"""

import argparse
import csv


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--last-frac", type=float, default=0.5)
    ap.add_argument("--top", type=int, default=15)
    a = ap.parse_args()
    rows = list(csv.DictReader(open(a.trace)))
    iv = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows)
    t0, t1 = iv[0][0], max(e for _, e, _ in iv)
    cut = t1 - (t1 - t0) * a.last_frac
    iv = [x for x in iv if x[0] >= cut]
    t0 = iv[0][0]
    busy = 0
    gaps = []
    cs, ce, last = iv[0][0], iv[0][1], iv[0][2]
    for s, e, n in iv[1:]:
        if s > ce:
            busy += ce - cs
            gaps.append((s - ce, last[:70], n[:70]))
            cs, ce, last = s, e, n
        elif e >= ce:
            ce, last = e, n
    busy += ce - cs
    span = ce - t0
    ksum = sum(e - s for s, e, _ in iv)
    print(
        f"window {span / 1e6:.2f} ms, GPU busy (union) {busy / 1e6:.2f} ms ({100 * busy / span:.1f}%), "
        f"sum of kernel times {ksum / 1e6:.2f} ms (overlap factor {ksum / max(busy, 1):.2f}), kernels {len(iv)}"
    )
    gaps.sort(reverse=True)
    print(f"idle {sum(g for g, _, _ in gaps) / 1e6:.2f} ms in {len(gaps)} gaps; largest:")
    for g, a_, b_ in gaps[: a.top]:
        print(f"  {g / 1e3:8.1f} us  after {a_}  before {b_}")


if __name__ == "__main__":
    main()
