"""Time the HIP 16-bit transpose (csrc/ops/transpose.hip) on the XL step's shapes; one JSON line of
us and GB/s per shape. CS336_TRANSPOSE=lds selects the previous LDS-tile kernel (read once).

    python scripts/transpose_bench.py
"""

import json
import os
import sys

import torch

sys.path.insert(0, __file__.rsplit("/scripts/", 1)[0])
from cs336_systems.ops._ext import ops  # noqa: E402

SHAPES = [(12288, 1600), (12800, 1600), (4800, 1600), (1600, 1600), (1600, 6400), (10000, 1600)]
res = {}
for R, C in SHAPES:
    x = torch.randn(R, C, device="cuda").bfloat16()
    y = ops().transpose2d(x)
    assert torch.equal(y, x.t().contiguous())
    for _ in range(3):
        ops().transpose2d(x)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    n = 50
    for _ in range(n):
        ops().transpose2d(x)
    e1.record()
    e1.synchronize()
    us = e0.elapsed_time(e1) * 1000 / n
    res[f"{R}x{C}"] = {"us": round(us, 2), "GBps": round(4 * R * C / us / 1e3, 1)}
print(json.dumps({"kernel": os.environ.get("CS336_TRANSPOSE", "reg"), "results": res}))
