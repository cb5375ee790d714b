"""FA2 forward / backward timing on the shapes that matter (for A/B runs of kernel variants via
env switches, one process per setting): BASELINE config 2 (B 4, H 16, N 4096, d 64/128, causal and
not), the XL step (B 24, H 25, N 512, d 64, causal) and the 2.7b step (B 12, H 32, N 1024, d 80).

    CS336_FA_DMA=0 python scripts/fa_ab.py ; CS336_FA_DMA=1 python scripts/fa_ab.py
    FA_AB_SHAPES="1,1,8192,128,0;1,1,4096,128,0" FA_AB_DTYPE=fp32 python scripts/fa_ab.py   # other shapes
"""

import json
import os
import sys

import torch

sys.path.insert(0, __file__.rsplit("/scripts/", 1)[0])
from cs336_systems import ops  # noqa: E402
from cs336_systems.utils.timing import do_bench  # noqa: E402

SHAPES = [(4, 16, 4096, 64, True), (4, 16, 4096, 64, False), (4, 16, 4096, 128, True), (4, 16, 4096, 128, False),
          (24, 25, 512, 64, True), (12, 32, 1024, 80, True)]
if os.environ.get("FA_AB_SHAPES"):
    SHAPES = [tuple(int(x) for x in sh.split(",")) for sh in os.environ["FA_AB_SHAPES"].split(";") if sh]
    SHAPES = [(B, H, N, D, bool(c)) for B, H, N, D, c in SHAPES]
DT = {"bf16": torch.bfloat16, "fp16": torch.float16, "fp32": torch.float32}[os.environ.get("FA_AB_DTYPE", "bf16")]
tag = {k: v for k, v in os.environ.items() if k.startswith("CS336_FA") or k == "FA_AB_DTYPE"}
for B, H, N, D, causal in SHAPES:
    torch.manual_seed(0)
    mk = lambda: torch.randn(B, N, H, D, device="cuda", dtype=DT).transpose(1, 2).requires_grad_(True)  # noqa: E731
    q, k, v = mk(), mk(), mk()
    do = torch.randn(B, H, N, D, device="cuda", dtype=DT)
    f = lambda: ops.FlashAttentionHIP.apply(q, k, v, causal)  # noqa: E731
    o = f()
    t_f = do_bench(f, quantiles=(0.5,))
    t_b = do_bench(lambda: torch.autograd.grad(o, (q, k, v), do, retain_graph=True), quantiles=(0.5,))
    fl = 4 * B * H * N * N * D * (0.5 if causal else 1.0)
    print(json.dumps(dict(env=tag, B=B, H=H, N=N, D=D, causal=causal, fwd_ms=round(t_f, 4), bwd_ms=round(t_b, 4),
                          fwd_tflops=round(fl / t_f / 1e9, 1), bwd_tflops=round(2.5 * fl / t_b / 1e9, 1))), flush=True)
