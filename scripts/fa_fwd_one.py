"""One FA2 shape, forward 5 times (for rocprofv3 --pmc passes on the forward kernel).
python scripts/fa_fwd_one.py B H N D causal"""
import sys

import torch

sys.path.insert(0, __file__.rsplit("/scripts/", 1)[0])
from cs336_systems import ops  # noqa: E402

B, H, N, D, causal = int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3]), int(sys.argv[4]), sys.argv[5] == "1"
torch.manual_seed(0)
mk = lambda: torch.randn(B, N, H, D, device="cuda", dtype=torch.bfloat16).transpose(1, 2)  # noqa: E731
q, k, v = mk(), mk(), mk()
for _ in range(5):
    ops.FlashAttentionHIP.apply(q, k, v, causal)
torch.cuda.synchronize()
print("done")
