"""Summarize a rocprofv3 --kernel-trace --stats CSV into per-step kernel time by category."""
import csv
import re
import sys

path = sys.argv[1]
steps = float(sys.argv[2]) if len(sys.argv) > 2 else 1.0
rows = list(csv.DictReader(open(path)))
cats = {}
def cat(n):
    if n.startswith("Cijk") or n.startswith("Custom_Cijk") or "gemm" in n.lower(): return "GEMM (hipBLASLt)"
    if "fa_fwd" in n: return "FA fwd"
    if "fa_bwd_dq" in n: return "FA bwd dq"
    if "fa_bwd_dkdv" in n: return "FA bwd dkdv"
    if "cs336" in n:
        m = re.search(r"(\w+_kernel)", n)
        return "cs336:" + (m.group(1) if m else n[:60])
    if "copy_kernel" in n or "bfloat16_copy" in n or "float32_copy" in n: return "dtype casts"
    if "add" in n.lower() and "at::native" in n: return "aten add"
    return "aten:" + n.split("(")[0][-60:]
tot = 0
for r in rows:
    c = cat(r["Name"]); t = float(r["TotalDurationNs"]) / 1e6 / steps
    cats.setdefault(c, [0.0, 0]); cats[c][0] += t; cats[c][1] += int(r["Calls"]); tot += t
for c, (t, n) in sorted(cats.items(), key=lambda x: -x[1][0])[:25]:
    print(f"{t:9.2f} ms/step {100*t/tot:5.1f}%  calls/step {n/steps:7.1f}  {c}")
print(f"{tot:9.2f} ms/step total kernel time")
