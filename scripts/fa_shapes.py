"""Run the HIP FA2 forward + backward a few times on the headline shapes (for rocprofv3 kernel
traces): seq 4096 (B 4, H 16, d 64/128, causal) and the XL training shape (B 24, H 25, N 512, d 64).

    rocprofv3 --kernel-trace --stats -- python scripts/fa_shapes.py
"""

import sys

import torch

sys.path.insert(0, __file__.rsplit("/scripts/", 1)[0])
from cs336_systems.ops.flash_attention import FlashAttentionHIP  # noqa: E402

SHAPES = [(4, 16, 4096, 64), (4, 16, 4096, 128), (24, 25, 512, 64)]
for B, H, N, D in SHAPES:
    torch.manual_seed(0)
    q, k, v = (torch.randn(B, H, N, D, device="cuda", dtype=torch.bfloat16, requires_grad=True) for _ in range(3))
    do = torch.randn(B, H, N, D, device="cuda", dtype=torch.bfloat16)
    for _ in range(5):
        o = FlashAttentionHIP.apply(q, k, v, True)
        torch.autograd.grad(o, (q, k, v), do)
    torch.cuda.synchronize()
    print(f"done {B}x{H}x{N}x{D}", flush=True)
