"""The XL step's attention backward in isolation, in the step's own layout (q/k/v strided views of
one fused QKV buffer, dQ/dK/dV into one fused dQKV buffer, RoPE inverse in the store) vs the
contiguous layout bench.flash times, to separate layout / RoPE-store costs from the kernel's.

    rocprofv3 --kernel-trace --stats -d gpurun_out/fa_layout -- python scripts/fa_step_layout.py
prints HIP-event ms per backward for each variant."""
import os
import sys

import torch

sys.path.insert(0, __file__.rsplit("/scripts/", 1)[0])
from cs336_systems import ops  # noqa: E402
from cs336_systems.models.fused import AttentionCore  # noqa: E402
from cs336_systems.models.transformer import RotaryEmbedding  # noqa: E402

B, H, N, D = (int(a) for a in (sys.argv[1:5] if len(sys.argv) > 4 else (48, 25, 512, 64)))
assert ops.load_ext(), ops.load_error()
torch.manual_seed(0)
rope = RotaryEmbedding(N, D, 10000.0, "cuda")
cos, sin = rope.cos.float().contiguous(), rope.sin.float().contiguous()


def timed(fn, reps=20):
    fn()
    torch.cuda.synchronize()
    flush = torch.empty(512 * 1024 * 1024 // 4, device="cuda")
    ts = []
    for _ in range(reps):
        flush.zero_()  # cold caches, as bench.flash
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        fn()
        e1.record()
        e1.synchronize()
        ts.append(e0.elapsed_time(e1))
    ts.sort()
    return ts[len(ts) // 2]


# step layout: fused qkv (B, N, 3*H*D), RoPE already applied (prerotated, as the QKV GEMM store does)
qkv = (torch.randn(B, N, 3 * H * D, device="cuda") * 0.5).to(torch.bfloat16).requires_grad_(True)
for rope_out in ("1", "0"):
    os.environ["CS336_FA_ROPE_OUT"] = rope_out
    o, _ = AttentionCore.apply(qkv, cos, sin, None, H, False, True)
    do = torch.randn_like(o)
    ms = timed(lambda: torch.autograd.grad(o, qkv, do, retain_graph=True))
    print(f"step layout, rope-out-in-FA={rope_out}: bwd {ms:.3f} ms")
# contiguous (B, H, N, D) layout without RoPE (bench.flash)
mk = lambda: torch.randn(B, H, N, D, device="cuda", dtype=torch.bfloat16).requires_grad_(True)  # noqa: E731
q, k, v = mk(), mk(), mk()
o = ops.FlashAttentionHIP.apply(q, k, v, True)
do = torch.randn_like(o)
ms = timed(lambda: torch.autograd.grad(o, (q, k, v), do, retain_graph=True))
print(f"contiguous (B,H,N,D), no RoPE: bwd {ms:.3f} ms")
# (B, N, H, D) memory viewed as (B, H, N, D) (the FA forward's own output layout), no RoPE
mk2 = lambda: torch.randn(B, N, H, D, device="cuda", dtype=torch.bfloat16).transpose(1, 2).requires_grad_(True)  # noqa: E731
q, k, v = mk2(), mk2(), mk2()
o = ops.FlashAttentionHIP.apply(q, k, v, True)
do = torch.randn_like(o)
ms = timed(lambda: torch.autograd.grad(o, (q, k, v), do, retain_graph=True))
print(f"(B,N,H,D) memory, no RoPE: bwd {ms:.3f} ms")
