"""Turn a ``CS336_GEMM_REPORT`` (bench.py --gemm best, per-problem candidate times) into the
committed selection table ``cs336_systems/tuning/gemm_table_mi355x.json`` (problem key -> pick).

    CS336_GEMM_TABLE=0 CS336_GEMM_REPORT=gpurun_out/rep.json python bench.py --steps 3 --warmup 2
    python scripts/gemm_table.py gpurun_out/rep.json [more reports ...] [--merge]

--merge keeps the committed table's entries for problems the given reports do not cover (e.g. adding
the shapes of another per-GPU batch).

With several reports (several boxes or runs) each problem takes the candidate with the lowest
median time over the reports, so one slow box or one noisy timing does not decide it.
"""

import json
import os
import statistics
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT = os.path.join(REPO, "cs336_systems", "tuning", "gemm_table_mi355x.json")


def main(paths):
    merge = "--merge" in paths
    paths = [p for p in paths if p != "--merge"]
    times: dict[str, dict[str, list[float]]] = {}
    for p in paths:
        for r in json.load(open(p)):
            for name, ms in r["ms"].items():
                if isinstance(ms, (int, float)):
                    times.setdefault(r["key"], {}).setdefault(name, []).append(float(ms))
    entries, detail = {}, {}
    for key, cands in times.items():
        med = {n: statistics.median(v) for n, v in cands.items()}
        best = min(med, key=med.get)
        # same 3 % tie rule as the runtime selection: hipBLASLt's default unless clearly beaten; and
        # the cs336 gemm8 kernel on a near-tie with any hipBLASLt pick (it has no stream-K
        # inter-workgroup waits and runs the same on every box)
        pick = best if "blas" not in med or med[best] < 0.97 * med["blas"] else "blas"
        if "g8" in med and pick != "g8" and med["g8"] <= 1.02 * med[pick]:
            pick = "g8"
        entries[key] = pick
        detail[key] = {n: round(v, 4) for n, v in med.items()}
    # Pinned regardless of timing: the XL vocabulary head (N or K = 10000 at d_model 1600) on the
    # cs336 gemm8 tail kernels, so the XL step runs no hipBLASLt stream-K kernel (rccl_env.py);
    # profiles/r4_gemm_report_xl_b96.json has the times (lm fwd 1.25 vs 1.09 ms, lm dX 1.36 vs 1.58 ms)
    for key in entries:
        if key.startswith("('nt'") and ("(10000, 1600)" in key or "(1600, 10000)" in key):
            entries[key] = "g8"
    # lt pins (hipBLASLt candidate index + kernel name per problem) from the first report that has them
    pins = []
    for p in paths:
        if os.path.exists(p + ".lt.json"):
            pins = json.load(open(p + ".lt.json"))
            break
    sources = [os.path.relpath(p, REPO) for p in paths]
    if merge:  # keep the committed table's other problems, pins and provenance; these reports add or override
        old = json.load(open(OUT))
        entries = {**old["entries"], **entries}
        detail = {**old["_meta"].get("median_ms", {}), **detail}
        have = {",".join(x.split(",", 6)[:6]) for x in pins}
        pins = pins + [x for x in old.get("lt_pins", []) if ",".join(x.split(",", 6)[:6]) not in have]
        sources = old["_meta"].get("sources", []) + sources
    if merge:  # pins apply to the kept entries too
        for key in entries:
            if key.startswith("('nt'") and ("(10000, 1600)" in key or "(1600, 10000)" in key):
                entries[key] = "g8"
    doc = {"_meta": {"sources": sources, "rule": "median ms over reports; blas unless beaten by > 3 %; "
                     "XL vocabulary head pinned to g8 (no stream-K kernel in the XL step)",
                     "median_ms": detail}, "entries": entries, "lt_pins": pins}
    with open(OUT, "w") as f:
        json.dump(doc, f, indent=1)
    print(f"{len(entries)} problems -> {OUT}")


if __name__ == "__main__":
    main(sys.argv[1:])
