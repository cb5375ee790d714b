"""hipBLASLt GEMMs of the projection shapes (torch.mm, bf16, hipBLASLt's default pick) for a
rocprofv3 kernel trace: with TENSILE_STREAMK_MAX_CUS set (bench.py / train.py set 248 at world size
> 1, cs336_systems/rccl_env.py) the stream-K grids must shrink to <= that many workgroups.

    rocprofv3 --kernel-trace --output-format csv -d gpurun_out/sk_cap -o run -- python scripts/streamk_cap_trace.py
    python scripts/streamk_cap_trace.py --summarize gpurun_out/sk_cap gpurun_out/sk_nocap
"""
import csv
import glob
import os
import sys


def run():
    import torch

    torch.manual_seed(0)
    for m, n, k in ((24576, 4800, 1600), (24576, 1600, 6400), (12288, 2560, 10240), (12288, 7680, 2560)):
        a = torch.randn(m, k, device="cuda", dtype=torch.bfloat16)
        b = torch.randn(k, n, device="cuda", dtype=torch.bfloat16)
        for _ in range(3):
            torch.mm(a, b)
    torch.cuda.synchronize()
    print("TENSILE_STREAMK_MAX_CUS", os.environ.get("TENSILE_STREAMK_MAX_CUS"))


def summarize(dirs):
    for d in dirs:
        rows = {}
        for f in glob.glob(f"{d}/**/*kernel_trace.csv", recursive=True):
            for r in csv.DictReader(open(f)):
                name = r["Kernel_Name"]
                if "Cijk" not in name and "Custom" not in name:
                    continue
                wg = int(r.get("Workgroup_Size_X") or r.get("Workgroup_Size") or 0)
                grid = int(r.get("Grid_Size_X") or r.get("Grid_Size") or 0)
                key = (name.split("_MT")[0][-40:] + "_MT" + name.split("_MT")[1][:12]) if "_MT" in name else name[:60]
                rows.setdefault(key, set()).add(grid // max(wg, 1))
        print(f"== {d}")
        for k, v in sorted(rows.items()):
            print(f"  workgroups {sorted(v)}  {k}")


if __name__ == "__main__":
    if len(sys.argv) > 1 and sys.argv[1] == "--summarize":
        summarize(sys.argv[2:])
    else:
        run()
