"""FlashAttention kernels with RoPE fused into the Q/K loads (and the inverse rotation fused into
the dQ/dK epilogues) vs an fp64 reference of rope -> attention, with and without explicit positions."""

import math

import pytest
import torch

from cs336_systems import ops
from cs336_systems.models import RotaryEmbedding
from cs336_systems.ops._ext import ops as _hip

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _ref(q, k, v, cos, sin, pos):
    qr = ops.rope_ref(q.double(), cos.double(), sin.double(), pos)
    kr = ops.rope_ref(k.double(), cos.double(), sin.double(), pos)
    s = qr @ kr.transpose(-1, -2) / math.sqrt(q.shape[-1])
    n = q.shape[-2]
    s = s.masked_fill(~torch.ones(n, n, dtype=torch.bool, device=q.device).tril(), float("-inf"))
    return torch.softmax(s, -1) @ v.double()


@pytest.mark.parametrize("D", [64, 128])
@pytest.mark.parametrize("with_pos", [False, True])
@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float32])
@pytest.mark.parametrize("N", [160, 512])  # 512: the split backward (dQ / dK rotated back by its reducers)
def test_fa_fused_rope(D, with_pos, dt, N):
    torch.manual_seed(0)
    B, H, ctx = 2, 3, max(256, N)
    re = RotaryEmbedding(ctx, D, 10000.0).to(DEV)
    cos, sin = re.cos.contiguous(), re.sin.contiguous()
    mk = lambda: torch.randn(B, N, H, D, device=DEV, dtype=dt).transpose(1, 2).requires_grad_(True)
    q, k, v = mk(), mk(), mk()
    pos = torch.randint(0, ctx, (B, N), device=DEV) if with_pos else None
    hip = _hip()
    o, lse = hip.fa_fwd(q, k, v, True, D**-0.5, cos, sin, pos)
    p = pos[:, None, :] if with_pos else torch.arange(N, device=DEV)
    qr, kr, vr = (t.detach().double().requires_grad_(True) for t in (q, k, v))
    o_ref = _ref(qr, kr, vr, cos, sin, p)
    tol = 3e-2 if dt == torch.bfloat16 else 2e-3
    torch.testing.assert_close(o.double(), o_ref, rtol=tol, atol=tol)
    do = torch.randn_like(o)
    dq, dk, dv = hip.fa_bwd(do, q, k, v, o, lse, True, D**-0.5, cos, sin, pos)
    o_ref.backward(do.double())
    gt = 6e-2 if dt == torch.bfloat16 else 5e-3
    for a, b in ((dq, qr.grad), (dk, kr.grad), (dv, vr.grad)):
        torch.testing.assert_close(a.double(), b, rtol=gt, atol=gt)
