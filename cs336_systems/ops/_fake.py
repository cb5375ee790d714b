"""Fake (meta) implementations of the ``torch.ops.cs336`` kernels so that ``torch.compile`` and
FakeTensor tracing see correct output shapes/dtypes/strides without running HIP code."""

from __future__ import annotations

import torch
from torch.library import register_fake


def _bnhd_like(q):
    B, H, N, D = q.shape
    return q.new_empty((B, N, H, D)).permute(0, 2, 1, 3)


@register_fake("cs336::fa_fwd")
def _fa_fwd(q, k, v, causal, scale, rope_cos=None, rope_sin=None, rope_pos=None):
    B, H, N, D = q.shape
    return _bnhd_like(q), q.new_empty((B, H, N), dtype=torch.float32)


@register_fake("cs336::fa_fwd_ot")
def _fa_fwd_ot(q, k, v, causal, scale):
    B, H, N, D = q.shape
    return _bnhd_like(q), q.new_empty((B, H, N), dtype=torch.float32), q.new_empty((H * D, B * N))


@register_fake("cs336::fa_bwd")
def _fa_bwd(do, q, k, v, o, lse, causal, scale, rope_cos=None, rope_sin=None, rope_pos=None):
    return _bnhd_like(q), _bnhd_like(k), _bnhd_like(v)


@register_fake("cs336::rmsnorm_fwd")
def _rms_fwd(x, w, eps, out_dtype):
    return x.new_empty(x.shape, dtype=out_dtype or x.dtype), x.new_empty((x.shape[0],), dtype=torch.float32)


@register_fake("cs336::rmsnorm_bwd")
def _rms_bwd(dy, x, w, rstd):
    return torch.empty_like(x), w.new_empty(w.shape, dtype=torch.float32)


@register_fake("cs336::rmsnorm_bwd_into")
def _rms_bwd_into(dy, x, w, rstd, dw_out):
    return torch.empty_like(x)


@register_fake("cs336::rmsnorm_bwd_add_into")
def _rms_bwd_add_into(dy, x, w, rstd, dres, emit_bf16, dw_out):
    return torch.empty_like(x), x.new_empty(x.shape if emit_bf16 else (0,), dtype=torch.bfloat16)


@register_fake("cs336::rmsnorm_bwd_add_t_into")
def _rms_bwd_add_t_into(dy, x, w, rstd, dres, emit_bf16, dw_out):
    dx2 = x.new_empty(x.shape if emit_bf16 else (0,), dtype=torch.bfloat16)
    return torch.empty_like(x), dx2, x.new_empty((x.shape[1], x.shape[0]), dtype=torch.bfloat16)


@register_fake("cs336::embedding_bwd")
def _emb_bwd(g, sorted_ids, perm, vocab):
    return g.new_empty((vocab, g.shape[1]), dtype=torch.float32)


@register_fake("cs336::cast_transpose_bf16")
def _cast_t(x):
    return x.new_empty(x.shape, dtype=torch.bfloat16), x.new_empty((x.shape[1], x.shape[0]), dtype=torch.bfloat16)


@register_fake("cs336::transpose2d")
def _transpose2d(x):
    return x.new_empty((x.shape[1], x.shape[0]))


@register_fake("cs336::gemm")
def _gemm(a, b, trans_a, trans_b, out_dtype, bm=0, bn=0, splits=0):
    M = a.shape[1] if trans_a else a.shape[0]
    N = b.shape[0] if trans_b else b.shape[1]
    return a.new_empty((M, N), dtype=out_dtype)


@register_fake("cs336::add_rmsnorm_fwd")
def _add_rms_fwd(x, r, w, eps, out_dtype):
    return torch.empty_like(x), x.new_empty(x.shape, dtype=out_dtype or x.dtype), x.new_empty((x.shape[0],), dtype=torch.float32)


@register_fake("cs336::rmsnorm_bwd_add")
def _rms_bwd_add(dy, x, w, rstd, dres, emit_bf16):
    dx2 = x.new_empty(x.shape if emit_bf16 else (0,), dtype=torch.bfloat16)
    return torch.empty_like(x), dx2, w.new_empty(w.shape, dtype=torch.float32)


@register_fake("cs336::rmsnorm_bwd_add_t")
def _rms_bwd_add_t(dy, x, w, rstd, dres, emit_bf16):
    dx2 = x.new_empty(x.shape if emit_bf16 else (0,), dtype=torch.bfloat16)
    dxt = x.new_empty((x.shape[1], x.shape[0]), dtype=torch.bfloat16)
    return torch.empty_like(x), dx2, dxt, w.new_empty(w.shape, dtype=torch.float32)


@register_fake("cs336::rope")
def _rope(x, cos, sin, pos, inverse):
    return _bnhd_like(x)


@register_fake("cs336::silu_mul_fwd")
def _sm_fwd(a, b):
    return torch.empty_like(a)


@register_fake("cs336::silu_mul_bwd")
def _sm_bwd(dh, a, b):
    return torch.empty_like(a), torch.empty_like(b)


@register_fake("cs336::xent_fwd")
def _xent_fwd(z, t):
    M = z.shape[0]
    return z.new_empty((M,), dtype=torch.float32), z.new_empty((M,), dtype=torch.float32)


@register_fake("cs336::xent_bwd")
def _xent_bwd(g, z, t, lse, mult):
    return torch.empty_like(z)


@register_fake("cs336::multi_tensor_l2norm")
def _l2(ts):
    return ts[0].new_empty((), dtype=torch.float32)


@register_fake("cs336::fa_bwd_into")
def _fa_bwd_into(do, q, k, v, o, lse, causal, scale, dq, dk, dv, rope_cos=None, rope_sin=None, rope_pos=None,
                 rope_out_only=False):
    return None


@register_fake("cs336::rope_into")
def _rope_into(x, cos, sin, pos, inverse, out):
    return None


if hasattr(torch.ops.cs336, "splitk_sum"):  # (absent from libraries built before round 5: A/B baselines)

    @register_fake("cs336::splitk_sum")
    def _splitk_sum(slabs, out, accumulate):
        return None


@register_fake("cs336::swiglu_fused_fwd")
def _swiglu_fused_fwd(y):
    return y.new_empty((*y.shape[:-1], y.shape[-1] // 2))


@register_fake("cs336::swiglu_fused_bwd")
def _swiglu_fused_bwd(dh, y):
    return torch.empty_like(y)


@register_fake("cs336::multi_tensor_cast_bf16")
def _cast_bf16(src, dst):
    return None
