"""RMSNorm: eager reference and the fused HIP kernel (``csrc/ops/rmsnorm.hip``).

Reference semantics (``cs336-basics/cs336_basics/model.py:101-107``): upcast to fp32,
``x * rsqrt(mean(x^2) + eps)``, multiply by the weight, cast back to the input dtype.

The HIP path fuses the whole row into one pass (one wave64 per row chunk, fp32 accumulate) and
can emit the normalized output directly in the autocast dtype (bf16), which removes the separate
cast kernel the eager path pays before every projection GEMM. Backward is one fused kernel for
``dx`` plus a two-stage column reduction for ``dw``.
"""

from __future__ import annotations

import torch

from ._ext import ops, use_hip


def rmsnorm_ref(x: torch.Tensor, weight: torch.Tensor, eps: float = 1e-5) -> torch.Tensor:
    in_dtype = x.dtype
    xf = x.to(torch.float32)
    rms = torch.rsqrt(xf.pow(2).mean(-1, keepdim=True) + eps)
    return (weight * (xf * rms)).to(in_dtype)


class RMSNormHIP(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, eps, out_dtype):
        shape = x.shape
        x2 = x.reshape(-1, shape[-1])
        if not x2.is_contiguous():
            x2 = x2.contiguous()
        y, rstd = ops().rmsnorm_fwd(x2, weight, eps, out_dtype)
        ctx.save_for_backward(x2, weight, rstd)
        ctx.shape = shape
        return y.view(*shape[:-1], shape[-1])

    @staticmethod
    def backward(ctx, dy):
        x2, weight, rstd = ctx.saved_tensors
        dy2 = dy.reshape(-1, dy.shape[-1])
        if not dy2.is_contiguous():
            dy2 = dy2.contiguous()
        dx, dw = ops().rmsnorm_bwd(dy2, x2, weight, rstd)
        return dx.view(ctx.shape), dw.to(weight.dtype), None, None


def rmsnorm(x: torch.Tensor, weight: torch.Tensor, eps: float = 1e-5, out_dtype: torch.dtype | None = None):
    """RMSNorm over the last dim. ``out_dtype`` defaults to the autocast dtype when autocast is on
    (the consumer is a GEMM that would cast anyway), else the input dtype."""
    H = x.shape[-1]
    if H % 4 == 0 and H <= 8192 and use_hip(x):
        if out_dtype is None:
            out_dtype = torch.get_autocast_dtype("cuda") if torch.is_autocast_enabled("cuda") else x.dtype
        return RMSNormHIP.apply(x, weight, eps, out_dtype)
    y = rmsnorm_ref(x, weight, eps)
    return y if out_dtype is None else y.to(out_dtype)
