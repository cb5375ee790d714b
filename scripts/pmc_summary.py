"""Summarize rocprofv3 --pmc / kernel-trace CSVs of one tag directory (scripts/fa_fwd_pmc.sh,
scripts/fa_bwd_pmc.sh layouts): per kernel-name substring, medians over dispatches of every counter,
wave-cycle fractions, VALU per MFMA and MFMA busy per SIMD-cycle (GRBM_GUI_ACTIVE / 8 = kernel cycles).

    python scripts/pmc_summary.py gpurun_out/fpmc_xl fa_fwd_kernel
"""
import csv
import glob
import statistics
import sys


def main(d, pat):
    vals, ts = {}, []
    for f in glob.glob(f"{d}/p*/**/*counter_collection.csv", recursive=True):
        per = {}
        for r in csv.DictReader(open(f)):
            if pat not in r["Kernel_Name"]:
                continue
            key = (r["Counter_Name"], r["Dispatch_Id"])
            per[key] = per.get(key, 0.0) + float(r["Counter_Value"])
        for (c, _), v in per.items():
            vals.setdefault(c, []).append(v)
    for f in glob.glob(f"{d}/kt/**/*kernel_trace.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if pat in r["Kernel_Name"]:
                ts.append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    m = {c: statistics.median(v) for c, v in vals.items()}
    out = {"us": round(statistics.median(ts), 1) if ts else None}
    wc = m.get("SQ_WAVE_CYCLES")
    for c in sorted(m):
        out[c] = m[c]
        if wc and c.startswith(("SQ_WAIT", "SQ_ACTIVE")):
            out[c + "/WAVE_CYCLES"] = round(m[c] / wc, 3)
    if "SQ_INSTS_VALU" in m and m.get("SQ_INSTS_MFMA"):
        out["valu_per_mfma"] = round(m["SQ_INSTS_VALU"] / m["SQ_INSTS_MFMA"], 2)
    if "GRBM_GUI_ACTIVE" in m and "SQ_VALU_MFMA_BUSY_CYCLES" in m:
        cyc = m["GRBM_GUI_ACTIVE"] / 8
        out["mfma_busy_per_simd_cycle"] = round(m["SQ_VALU_MFMA_BUSY_CYCLES"] / (cyc * 1024), 3)
        if ts:
            out["clock_ghz"] = round(cyc / (statistics.median(ts) * 1e3), 2)
    for k, v in out.items():
        print(f"{k:40s} {v}")


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else "")
