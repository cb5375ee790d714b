#!/bin/bash
# kernel trace of the XL step with the dW GEMMs on a side stream (batch 48): which kernels slow down
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out; rm -rf gpurun_out/dwsprof
CS336_DW_STREAM=1 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/dwsprof -o run -- python bench.py --batch 48 --steps 2 --warmup 2 > gpurun_out/dwsprof.log 2>&1 || { tail -20 gpurun_out/dwsprof.log; exit 1; }
T=$(find gpurun_out/dwsprof -name '*kernel_trace.csv' | head -n1)
python - "$T" <<'P'
import csv, sys, collections
rows = list(csv.DictReader(open(sys.argv[1])))
iv = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"], r.get("Stream_Id", ""), r.get("Queue_Id", "")) for r in rows)
starts = [s for s, _, n, _, _ in iv if "vectorized_gather_kernel" in n]
lo, hi = starts[-2], starts[-1]
step = [x for x in iv if lo <= x[0] < hi]
print("step window ms", (hi - lo) / 1e6, "kernels", len(step))
agg = collections.defaultdict(lambda: [0, 0.0])
for s, e, n, st, q in step:
    k = (n.split("(")[0][:60], st, q)
    agg[k][0] += 1
    agg[k][1] += (e - s) / 1e6
for k, (c, t) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:15]:
    print(f"{t:9.2f} ms {c:5d}  stream {k[1]} queue {k[2]}  {k[0]}")
# busy time (union of kernel intervals) vs window
busy, cur_s, cur_e = 0, None, None
for s, e, *_ in step:
    if cur_e is None or s > cur_e:
        if cur_e is not None: busy += cur_e - cur_s
        cur_s, cur_e = s, e
    else:
        cur_e = max(cur_e, e)
busy += cur_e - cur_s
print("union of kernel time ms", busy / 1e6)
P
