"""Summarize `scripts/ab.py bench` JSON lines (gpurun_out/ab_bench_<label>_<round>.log): ms/step,
tokens/s, peak memory, median shader clock and board power per arm and round."""

import glob
import json
import sys

pat = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/ab_bench_*_*.log"
for f in sorted(glob.glob(pat)):
    for line in open(f):
        if line.startswith("{") and '"ms_per_step"' in line:
            d = json.loads(line)
            c = d.get("gpu_clocks") or {}
            print(f, d["ms_per_step"], d["value"], d.get("peak_mem_gib"),
                  (c.get("sclk_mhz") or {}).get("median"), (c.get("power_w") or {}).get("median"))
