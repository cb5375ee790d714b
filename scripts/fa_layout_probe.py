"""FA2 forward / backward at B 4 H 16 N 4096 on three input layouts: (B, N, H, d) transposed views
(the model's), contiguous (B, H, N, d) (bench.flash's), and (B, H, N + pad, d) sliced (contiguous
heads whose starts are not a power-of-two apart). Tests whether a layout gap is DRAM channel
camping (heads 512 KiB apart, blocks at the same key tile) or something else.
    python scripts/fa_layout_probe.py"""

import json
import sys

import torch

sys.path.insert(0, __file__.rsplit("/scripts/", 1)[0])
from cs336_systems import ops  # noqa: E402
from cs336_systems.utils.timing import do_bench  # noqa: E402

B, H, N = 4, 16, 4096
for D in (64, 128):
    for causal in (True, False):
        for layout in ("bnhd", "bhnd", "bhnd_pad"):
            torch.manual_seed(0)
            if layout == "bnhd":
                mk = lambda: torch.randn(B, N, H, D, device="cuda", dtype=torch.bfloat16).transpose(1, 2)  # noqa: E731
            elif layout == "bhnd":
                mk = lambda: torch.randn(B, H, N, D, device="cuda", dtype=torch.bfloat16)  # noqa: E731
            else:
                mk = lambda: torch.randn(B, H, N + 40, D, device="cuda", dtype=torch.bfloat16)[:, :, :N]  # noqa: E731
            q, k, v = (mk().requires_grad_(True) for _ in range(3))
            do = torch.randn(B, H, N, D, device="cuda", dtype=torch.bfloat16)
            with torch.no_grad():
                tf = do_bench(lambda: ops.FlashAttentionHIP.apply(q, k, v, causal), quantiles=(0.5,))
            o = ops.FlashAttentionHIP.apply(q, k, v, causal)
            tb = do_bench(lambda: torch.autograd.grad(o, (q, k, v), do, retain_graph=True), quantiles=(0.5,))
            fl = 4 * B * H * N * N * D * (0.5 if causal else 1.0)
            print(json.dumps(dict(D=D, causal=causal, layout=layout, fwd_tf=round(fl / tf / 1e9, 1),
                                  bwd_tf=round(2.5 * fl / tb / 1e9, 1))), flush=True)
