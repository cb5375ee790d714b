"""Median time per FlashAttention kernel instantiation and grid in a rocprofv3 kernel trace."""
import csv
import sys
from collections import defaultdict

agg = defaultdict(list)
for r in csv.DictReader(open(sys.argv[1])):
    n = r["Kernel_Name"]
    if "fa_" not in n:
        continue
    g = int(r["Grid_Size_X"]) // int(r["Workgroup_Size_X"])
    agg[(n.split("(")[0].split("fa::")[-1], g)].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
for (name, g), v in agg.items():
    v = sorted(v)
    print(f"{name:48s} wgs {g:6d} n={len(v)} median {v[len(v) // 2]:8.1f} us")
