"""One FA2 shape, forward once then backward 5 times (for rocprofv3 --pmc passes on the backward
kernels).  python scripts/fa_bwd_one.py B H N D causal"""
import sys

import torch

sys.path.insert(0, __file__.rsplit("/scripts/", 1)[0])
from cs336_systems import ops  # noqa: E402

B, H, N, D, causal = int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3]), int(sys.argv[4]), sys.argv[5] == "1"
torch.manual_seed(0)
mk = lambda: torch.randn(B, N, H, D, device="cuda", dtype=torch.bfloat16).transpose(1, 2).requires_grad_(True)  # noqa: E731
q, k, v = mk(), mk(), mk()
o = ops.FlashAttentionHIP.apply(q, k, v, causal)
do = torch.randn_like(o)
for _ in range(5):
    torch.autograd.grad(o, (q, k, v), do, retain_graph=True)
torch.cuda.synchronize()
print("done")
