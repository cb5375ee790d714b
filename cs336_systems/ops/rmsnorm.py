"""RMSNorm: eager reference and the fused HIP kernel (``csrc/ops/rmsnorm.hip``).

Reference semantics (``cs336-basics/cs336_basics/model.py:101-107``): upcast to fp32,
``x * rsqrt(mean(x^2) + eps)``, multiply by the weight, cast back to the input dtype.

The HIP path fuses the whole row into one pass (one wave64 per row chunk, fp32 accumulate) and
can emit the normalized output directly in the autocast dtype (bf16), which removes the separate
cast kernel the eager path pays before every projection GEMM. Backward is one fused kernel for
``dx`` plus a two-stage column reduction for ``dw``.
"""

from __future__ import annotations

import os

import torch

from ._ext import ops, use_hip


def rmsnorm_ref(x: torch.Tensor, weight: torch.Tensor, eps: float = 1e-5) -> torch.Tensor:
    in_dtype = x.dtype
    xf = x.to(torch.float32)
    rms = torch.rsqrt(xf.pow(2).mean(-1, keepdim=True) + eps)
    return (weight * (xf * rms)).to(in_dtype)


def _dw_target(weight) -> torch.Tensor | None:
    """The DDP bucket view to write the weight gradient into (``parallel/ddp.py`` sets
    ``_cs336_grad_out``), when the gradient is unset and fp32: the column reduction writes it there
    and autograd adopts an alias of it as ``.grad``, so the bucket needs no copy of it (the GEMMs'
    dW does the same, ``models/fused.py``)."""
    t = getattr(weight, "_cs336_grad_out", None)
    if t is None or weight.grad is not None or t.dtype != torch.float32 or not t.is_contiguous():
        return None
    return t if t.shape == weight.shape else None


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
        ctx.wparam = weight
        return y.view(*shape[:-1], shape[-1])

    @staticmethod
    def backward(ctx, dy):
        x2, weight, rstd = ctx.saved_tensors
        dy2 = dy.reshape(-1, dy.shape[-1])
        if not dy2.is_contiguous():
            dy2 = dy2.contiguous()
        tgt = _dw_target(ctx.wparam) if ctx.needs_input_grad[1] else None
        if tgt is not None:
            dx = ops().rmsnorm_bwd_into(dy2, x2, weight, rstd, tgt)
            return dx.view(ctx.shape), tgt.view_as(tgt), None, None
        dx, dw = ops().rmsnorm_bwd(dy2, x2, weight, rstd)
        return dx.view(ctx.shape), dw.to(weight.dtype), None, None


class AddRMSNormHIP(torch.autograd.Function):
    """``s = x + r; y = rmsnorm(s)`` in one pass; backward ``ds = rmsnorm_bwd(dy) + ds_next`` in one
    pass, emitting the bf16 copy of ``ds`` for a bf16 branch ``r`` from the same kernel."""

    @staticmethod
    def forward(ctx, x, r, weight, eps, out_dtype):
        shape = x.shape
        s, y, rstd = ops().add_rmsnorm_fwd(x.reshape(-1, shape[-1]), r.reshape(-1, shape[-1]), weight, eps, out_dtype)
        ctx.save_for_backward(s, weight, rstd)
        ctx.shape, ctx.r_dtype = shape, r.dtype
        ctx.wparam = weight
        return s.view(shape), y.view(*shape[:-1], y.shape[-1])

    @staticmethod
    def backward(ctx, ds, dy):
        s, weight, rstd = ctx.saved_tensors
        H = ctx.shape[-1]
        if dy is None:
            dx = ds
            dw = torch.zeros_like(weight)
            dr = ds.to(ctx.r_dtype)
            return dx, dr, dw, None, None
        dy2 = dy.reshape(-1, H)
        if not dy2.is_contiguous():
            dy2 = dy2.contiguous()
        # dw straight into the DDP bucket view when there is one (no adopt copy)
        tgt = _dw_target(ctx.wparam) if ctx.needs_input_grad[2] else None
        if ds is None:
            if tgt is not None:
                dx, dw = ops().rmsnorm_bwd_into(dy2, s, weight, rstd, tgt), tgt
            else:
                dx, dw = ops().rmsnorm_bwd(dy2, s, weight, rstd)
            dr = dx if ctx.r_dtype == dx.dtype else dx.to(ctx.r_dtype)
        else:
            ds2 = ds.reshape(-1, H)
            if not ds2.is_contiguous() or ds2.dtype != s.dtype:
                ds2 = ds2.contiguous().to(s.dtype)
            emit = ctx.r_dtype == torch.bfloat16 and s.dtype != torch.bfloat16
            if emit and _want_transposed_grad(s):
                # the branch is a narrow projection whose dW takes dYᵀ (models/fused.py): write it
                # here, transposed through LDS, instead of a separate transpose of dr
                if tgt is not None:
                    dx, dx_bf16, dxt = ops().rmsnorm_bwd_add_t_into(dy2, s, weight, rstd, ds2, True, tgt)
                    dw = tgt
                else:
                    dx, dx_bf16, dxt, dw = ops().rmsnorm_bwd_add_t(dy2, s, weight, rstd, ds2, True)
                from ..models.fused import offer_transposed_grad

                offer_transposed_grad(dx_bf16, dxt)
            elif tgt is not None:
                dx, dx_bf16 = ops().rmsnorm_bwd_add_into(dy2, s, weight, rstd, ds2, emit, tgt)
                dw = tgt
            else:
                dx, dx_bf16, dw = ops().rmsnorm_bwd_add(dy2, s, weight, rstd, ds2, emit)
            dr = dx_bf16 if emit else (dx if ctx.r_dtype == dx.dtype else dx.to(ctx.r_dtype))
        # a fresh alias of the bucket view: AccumulateGrad adopts it as .grad without a copy
        dw = dw.view_as(dw) if tgt is not None else dw.to(weight.dtype)
        return dx.view(ctx.shape), dr.view(ctx.shape), dw, None, None


# CS336_DYT_FUSED=1: the fused kernel (LDS-staged transposed store) measured 90 us per call vs
# 60 + 15 us for the row-major kernel plus a separate transpose on XL (-0.5 ms/step), so the
# two-kernel path is the default. Read once at import (the backward is traced by torch.compile).
_DYT_FUSED = os.environ.get("CS336_DYT", "1") != "0" and os.environ.get("CS336_DYT_FUSED", "0") != "0"


def _want_transposed_grad(s: torch.Tensor) -> bool:
    H, M = s.shape[-1], s.numel() // s.shape[-1]
    if not _DYT_FUSED:
        return False
    rows = 16 if H * 36 <= 65536 else 8
    return s.is_cuda and H % 8 == 0 and H <= 8192 and M % rows == 0


def add_rmsnorm_ref(x, r, weight, eps=1e-5):
    s = x + r
    return s, rmsnorm_ref(s, weight, eps)


def add_rmsnorm(x: torch.Tensor, r: torch.Tensor, weight: torch.Tensor, eps: float = 1e-5, out_dtype: torch.dtype | None = None):
    """Pre-norm residual step: returns ``(s, rmsnorm(s))`` with ``s = x + r`` (reference
    ``model.py:380-386`` does the add and the next block's norm as two ops)."""
    H = x.shape[-1]
    if (
        H % 4 == 0
        and H <= 8192
        and use_hip(x)
        and weight.dtype == torch.float32
        and x.dtype in (torch.float32, torch.bfloat16)
        and r.dtype in (torch.float32, torch.bfloat16)
        and x.shape == r.shape
        and (x.dtype == torch.float32 or r.dtype == x.dtype)  # x + r stays in x's dtype (traceable form)
    ):
        if out_dtype is None:
            out_dtype = torch.get_autocast_dtype("cuda") if torch.is_autocast_enabled("cuda") else x.dtype
        if not x.is_contiguous():
            x = x.contiguous()
        if not r.is_contiguous():
            r = r.contiguous()
        return AddRMSNormHIP.apply(x, r, weight, eps, out_dtype)
    s = x + r
    return s, rmsnorm(s, weight, eps, out_dtype)


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
