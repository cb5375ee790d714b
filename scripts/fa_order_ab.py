"""Time causal HIP FA2 fwd+bwd on shapes whose batch*heads is / is not a multiple of 8 (one process per
CS336_FA_ORDER value, the switch is read once): prints one JSON line of median ms per shape.

    CS336_FA_ORDER=2 python scripts/fa_order_ab.py
"""

import json
import os
import sys

import torch

sys.path.insert(0, __file__.rsplit("/scripts/", 1)[0])
from cs336_systems.ops.flash_attention import FlashAttentionHIP  # noqa: E402

SHAPES = [(3, 25, 4096, 64), (5, 25, 512, 64), (24, 25, 512, 64), (4, 12, 2048, 64), (2, 20, 4096, 128), (4, 16, 4096, 128)]
if len(sys.argv) > 1:  # shapes as B,H,N,D ...
    SHAPES = [tuple(int(x) for x in a.split(",")) for a in sys.argv[1:]]
res = {}
for B, H, N, D in SHAPES:
    torch.manual_seed(0)
    q, k, v = (torch.randn(B, N, H, D, device="cuda", dtype=torch.bfloat16).transpose(1, 2).requires_grad_() for _ in range(3))
    do = torch.randn(B, H, N, D, device="cuda", dtype=torch.bfloat16)
    ts = []
    for i in range(15):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        o = FlashAttentionHIP.apply(q, k, v, True)
        torch.autograd.grad(o, (q, k, v), do)
        e1.record()
        e1.synchronize()
        if i >= 3:
            ts.append(e0.elapsed_time(e1))
    ts.sort()
    res[f"{B}x{H}x{N}x{D} nbh%8={B * H % 8}"] = round(ts[len(ts) // 2], 4)
print(json.dumps({"order": os.environ.get("CS336_FA_ORDER", "1"), "median_ms": res}))
