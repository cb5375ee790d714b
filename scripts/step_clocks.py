"""Per-role clock and MFMA occupancy of the kernels of ONE training step, from a rocprofv3 run with
--kernel-trace and --pmc GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES over bench.py
(`bash scripts/pmc_step_clocks.sh`). The effective clock of a dispatch is GRBM_GUI_ACTIVE / 8 (the
counter sums the 8 XCDs) over its duration (MI355X_MICROARCH.md, DVFS give-back); MFMA busy is
SQ_VALU_MFMA_BUSY_CYCLES per SIMD-cycle (1,024 SIMDs). GEMM roles follow the step's launch order
(scripts/roofline_table.py).

    python scripts/step_clocks.py gpurun_out/stepclk [--layers 48]
"""

import argparse
import csv
import glob
import statistics
from collections import defaultdict

from roofline_table import is_gemm


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--layers", type=int, default=48)
    a = ap.parse_args()
    kt = [r for f in glob.glob(f"{a.dir}/**/*kernel_trace.csv", recursive=True) for r in csv.DictReader(open(f))]
    cnt = defaultdict(dict)
    for f in glob.glob(f"{a.dir}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            d = cnt[r["Dispatch_Id"]]
            d[r["Counter_Name"]] = d.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    iv = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"], r["Dispatch_Id"]) for r in kt)
    starts = [s for s, _, n, _ in iv if "vectorized_gather_kernel" in n]
    lo, hi = starts[-2], starts[-1]
    step = [x for x in iv if lo <= x[0] < hi]
    xf = [s for s, _, k, _ in step if "xent_fwd" in k][0]
    g = [x for x in step if is_gemm(x[2])]
    fwd = [x for x in g if x[0] < xf]
    bwd = [x for x in g if x[0] >= xf]
    role = {}
    L = a.layers
    if len(fwd) == 4 * L + 1 and len(bwd) == 8 * L + 2:
        for i, x in enumerate(fwd[:-1]):
            role[x[3]] = ("qkv", "o", "w13", "w2")[i % 4] + " fwd"
        role[fwd[-1][3]] = "lm fwd"
        order = ["w2 dW", "w2 dX", "w13 dX", "w13 dW", "o dX", "o dW", "qkv dX", "qkv dW"]
        lm = ("dX", "dW")
        if "gemm8w" in bwd[0][2] and "gemm8w" not in bwd[1][2]:
            lm = ("dW", "dX")
        for j, x in enumerate(bwd):
            role[x[3]] = "lm " + lm[j] if j < 2 else order[(j - 2) % 8]
    rows = defaultdict(list)
    for s, e, k, d in step:
        c = cnt.get(d)
        if not c or "GRBM_GUI_ACTIVE" not in c:
            continue
        name = role.get(d) or ("FA fwd" if "fa_fwd" in k else "FA bwd" if "fa_bwd" in k else k.split("(")[0].split("<")[0][-40:])
        us = (e - s) / 1e3
        cyc = c["GRBM_GUI_ACTIVE"] / 8
        busy = c.get("SQ_VALU_MFMA_BUSY_CYCLES", 0.0) / (cyc * 1024) if cyc else 0.0
        rows[name].append((us, cyc / (us * 1e3), busy))
    print("| kernel (role) | calls | median us | clock GHz | MFMA busy per SIMD-cycle |")
    print("|---|---|---|---|---|")
    for name, v in sorted(rows.items(), key=lambda kv: -sum(x[0] for x in kv[1])):
        if sum(x[0] for x in v) < 300:
            continue
        print(f"| {name} | {len(v)} | {statistics.median(x[0] for x in v):.1f} | "
              f"{statistics.median(x[1] for x in v):.2f} | {statistics.median(x[2] for x in v):.3f} |")


if __name__ == "__main__":
    main()
