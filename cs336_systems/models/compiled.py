"""The fused Transformer stages as ``torch.library`` custom ops, for ``torch.compile(model)``.

The eager fast path (``models/fused.py``) is a set of ``torch.autograd.Function``s whose Python
reads bf16 / Wᵀ weight shadows, DDP bucket targets, side streams and producer offers keyed by data
pointers -- all of which Dynamo cannot trace (each one a graph break). Here the same kernels run
behind opaque, functional custom ops (fake impls give Dynamo/AOTAutograd the shapes; the eager impls
run the HIP path), each forward op paired with a backward op through ``register_autograd``:

============================  =====================================================  ==============================
op                            forward                                                backward
============================  =====================================================  ==============================
``cs336c::linear``            ``x @ [W_0; W_1; ...]ᵀ`` (gemm8 / table pick)           ``linear_bwd``: dX by gemm8 on the
                                                                                     Wᵀ shadow, fp32 dW by gemm8w
``cs336c::qkv_rope``          fused QKV GEMM with RoPE on q|k in the store (epi 3)   ``linear_bwd``
``cs336c::attn``              causal FA2 forward on the strided q / k / v views     ``attn_bwd``: FA2 backward into
                                                                                     one d(qkv), dQ/dK rotated back
``cs336c::swiglu_ffn``        W1|W3 GEMM + SwiGLU epilogue, then W2 (gemm8 epi 1)    ``swiglu_ffn_bwd``: dW2, the W2
                                                                                     input grad with the SwiGLU
                                                                                     backward epilogue (epi 2), dX, dW13
============================  =====================================================  ==============================

The ops receive the ``nn.Parameter`` objects themselves (``torch.compile`` hands the module's real
parameters to an opaque op), so the bf16 / Wᵀ shadows that the fused AdamW writes are used exactly
as in eager mode, with the same ``_version`` validity check. Weight gradients come back as one fp32
tensor per group and are split into the per-parameter gradients by the traced backward formula (a
view, no copy). The norms, the residual adds, the embedding and the loss are already traceable
(``ops/rmsnorm.py``, ``ops/cross_entropy.py``: autograd Functions over ``torch.ops.cs336`` kernels
with fake impls, ``ops/_fake.py``).

On CPU every op runs the eager reference math, which is what the CPU tests of this module check
against (``tests/test_compile_path.py``); the GPU test checks zero graph breaks and the gradients
of the compiled XL-shape step against eager (``tests/test_compile_gpu.py``).

Reference: the student benchmark compiles the whole model (``cs336_systems/benchmark.py:43-44``,
sweep ``:280-282``) and the attention module (``benchmark_attention.py:45,134``).
"""

from __future__ import annotations

from typing import List, Optional, Tuple

import torch
from torch import Tensor

from ..ops import gemm
from ..ops._ext import ops as _hip
from ..ops.rope import rope_ref
from . import fused

_BF16 = torch.bfloat16


def _cast(t: Tensor, dt: torch.dtype) -> Tensor:
    return t if t.dtype == dt else t.to(dt)


def _hip_ok(t: Tensor) -> bool:
    from ..ops import use_hip

    return t.is_cuda and use_hip(t)


# ------------------------------------------------------------------------------------------
# linear (and the QKV projection with RoPE in its store)
# ------------------------------------------------------------------------------------------
def _weights(ws: List[Tensor], cdt: torch.dtype) -> Tuple[Tensor, Tensor]:
    """(W, Wᵀ) in ``cdt`` for a group of weights: the forward's compute weight and the K-major
    operand the backward's input-gradient GEMM reads. With valid bf16 / Wᵀ shadows (the fused AdamW
    writes them) both are views of the shadows; without them one HIP pass casts the fp32 master and
    writes its transpose (``cast_transpose_bf16``: 8 B per element, where the eager path's cast plus
    transpose move 10) -- and the backward never re-casts: Wᵀ is saved from the forward."""
    ws = list(ws)
    if cdt == _BF16 and all(fused.shadow_valid(p) for p in ws):
        w = fused.compute_weight(ws, cdt)  # the shadow view
        wt = fused.compute_weight_t(ws)
        return w, wt if wt is not None else (fused._transpose(w) if w.is_cuda else w.t().contiguous())
    if cdt == _BF16:
        g = fused.grouped_view(ws) if len(ws) > 1 else ws[0].detach()
        if (g is not None and g.dtype == torch.float32 and _hip_ok(g) and g.dim() == 2 and g.stride(1) == 1
                and g.shape[0] % 8 == 0 and g.shape[1] % 8 == 0 and g.stride(0) % 4 == 0 and g.data_ptr() % 16 == 0):
            return _hip().cast_transpose_bf16(g)
    w = fused.compute_weight(ws, cdt)
    return w, (fused._transpose(w) if w.is_cuda else w.t().contiguous())


@torch.library.custom_op("cs336c::linear", mutates_args=())
def _linear(x2: Tensor, ws: List[Tensor], cdt: torch.dtype) -> Tuple[Tensor, Tensor]:
    """(``x2 @ [W_0; W_1; ...]ᵀ`` in ``cdt``, Wᵀ) -- ``cdt`` is the autocast dtype or the weights'."""
    w, wt = _weights(ws, cdt)
    x = _cast(x2, cdt)
    if _hip_ok(x):
        return gemm.mm_nt(x, w), wt
    return x @ w.t(), wt


@_linear.register_fake
def _linear_fake(x2, ws, cdt):
    rows, k = sum(w.shape[0] for w in ws), ws[0].shape[1]
    return x2.new_empty((x2.shape[0], rows), dtype=cdt), x2.new_empty((k, rows), dtype=cdt)


def linear(x2: Tensor, ws: List[Tensor], cdt: torch.dtype) -> Tensor:
    return _linear(x2, ws, cdt)[0]


@torch.library.custom_op("cs336c::linear_bwd", mutates_args=())
def linear_bwd(dy: Tensor, x2: Tensor, wt: Tensor, cdt: torch.dtype, need_dx: bool) -> Tuple[Tensor, Tensor]:
    """(dX, fp32 dW) of :func:`linear` from the forward's saved Wᵀ; dX is an empty tensor when not
    needed."""
    dy = _cast(dy, cdt)
    x = _cast(x2, cdt)
    dx = dy.new_empty((0,))
    if need_dx:
        dx = gemm.mm_nt(dy, wt) if _hip_ok(dy) else dy @ wt.t()
    if _hip_ok(dy) and dy.dtype == _BF16 and gemm.dw_g8w_ok(dy, x):
        dw = gemm.mm_dw(dy, x)
    elif _hip_ok(dy) and dy.dtype == _BF16:
        dw = gemm.mm_tn_fp32(dy, x)
    else:
        dw = dy.t().float() @ x.float()
    return dx, dw


@linear_bwd.register_fake
def _linear_bwd_fake(dy, x2, wt, cdt, need_dx):
    dx = dy.new_empty((x2.shape[0], x2.shape[1]) if need_dx else (0,), dtype=cdt)
    return dx, dy.new_empty((wt.shape[1], x2.shape[1]), dtype=torch.float32)


def _linear_setup(ctx, inputs, output):
    x2, ws, cdt = inputs[0], inputs[1], inputs[2]
    _, wt = output
    ctx.mark_non_differentiable(wt)
    ctx.save_for_backward(x2, wt)
    ctx.cdt, ctx.rows = cdt, [w.shape[0] for w in ws]
    ctx.wdtypes = [w.dtype for w in ws]
    ctx.x_dtype = x2.dtype


def _linear_grads(ctx, g: Tensor):
    x2, wt = ctx.saved_tensors
    need_dx = ctx.needs_input_grad[0]
    dx, dw = linear_bwd(g, x2, wt, ctx.cdt, need_dx)
    parts = [p if p.dtype == dt else p.to(dt) for p, dt in zip(dw.split(ctx.rows, 0), ctx.wdtypes)]
    return (_cast(dx, ctx.x_dtype) if need_dx else None), parts


def _linear_backward(ctx, g, _gwt):
    dx, parts = _linear_grads(ctx, g)
    return dx, parts, None


_linear.register_autograd(_linear_backward, setup_context=_linear_setup)


@torch.library.custom_op("cs336c::qkv_rope", mutates_args=())
def _qkv_rope(x2: Tensor, ws: List[Tensor], cos: Tensor, sin: Tensor, seq: int, n_heads: int) -> Tuple[Tensor, Tensor]:
    """(fused QKV projection ``x2 @ [Wq; Wk; Wv]ᵀ`` (bf16) with RoPE applied to its q|k columns, Wᵀ);
    rows of ``x2`` are tokens ``row % seq`` of their sequence."""
    w, wt = _weights(ws, _BF16)
    x = _cast(x2, _BF16)
    dk = ws[0].shape[0] // n_heads
    rope_cols = 2 * n_heads * dk
    if _hip_ok(x) and dk <= 96 and gemm.gemm8_ok(x, w, 3, rope_cols):
        return gemm.gemm8_rope(x, w, cos, sin, None, seq, rope_cols, dk), wt
    y = gemm.mm_nt(x, w) if _hip_ok(x) else x @ w.t()
    B = x.shape[0] // seq
    qk = y.view(B, seq, 3, n_heads, dk)[:, :, 0:2].reshape(B, seq, 2 * n_heads, dk).transpose(1, 2)
    pos = torch.arange(seq, device=x.device)
    rot = rope_ref(qk, cos, sin, pos)  # (B, 2H, seq, dk)
    y.view(B, seq, 3, n_heads, dk)[:, :, 0:2].copy_(rot.transpose(1, 2).reshape(B, seq, 2, n_heads, dk))
    return y, wt


@_qkv_rope.register_fake
def _qkv_rope_fake(x2, ws, cos, sin, seq, n_heads):
    rows, k = sum(w.shape[0] for w in ws), ws[0].shape[1]
    return x2.new_empty((x2.shape[0], rows), dtype=_BF16), x2.new_empty((k, rows), dtype=_BF16)


def qkv_rope(x2: Tensor, ws: List[Tensor], cos: Tensor, sin: Tensor, seq: int, n_heads: int) -> Tensor:
    return _qkv_rope(x2, ws, cos, sin, seq, n_heads)[0]


def _qkv_setup(ctx, inputs, output):
    _linear_setup(ctx, (inputs[0], inputs[1], _BF16), output)


def _qkv_backward(ctx, g, _gwt):
    # g is w.r.t. the un-rotated projection output (attn_bwd rotates dQ/dK back)
    dx, parts = _linear_grads(ctx, g)
    return dx, parts, None, None, None, None


_qkv_rope.register_autograd(_qkv_backward, setup_context=_qkv_setup)


# ------------------------------------------------------------------------------------------
# attention core on the fused (rotated) QKV layout
# ------------------------------------------------------------------------------------------
def _split(qkv: Tensor, n_heads: int):
    B, N, three_d = qkv.shape
    dk = three_d // (3 * n_heads)
    t5 = qkv.view(B, N, 3, n_heads, dk)
    qk = t5[:, :, 0:2].reshape(B, N, 2 * n_heads, dk).transpose(1, 2)
    return qk[:, :n_heads], qk[:, n_heads:], t5[:, :, 2].transpose(1, 2)


@torch.library.custom_op("cs336c::attn", mutates_args=())
def attn(qkv: Tensor, cos: Tensor, sin: Tensor, n_heads: int) -> Tuple[Tensor, Tensor]:
    """Causal attention over a fused ``(B, N, 3·H·dk)`` projection whose q|k are already rotated;
    returns ``o`` as a ``(B, H, N, dk)`` view of ``(B, N, H, dk)`` memory and the (B, H, N) LSE.
    (``cos``/``sin`` are for the backward's inverse rotation of dQ/dK.)"""
    q, k, v = _split(qkv, n_heads)
    if _hip_ok(qkv):
        return _hip().fa_fwd(q, k, v, True, q.shape[-1] ** -0.5)
    qf, kf, vf = q.float(), k.float(), v.float()
    s = qf @ kf.transpose(-1, -2) * q.shape[-1] ** -0.5
    N = q.shape[2]
    s = s.masked_fill(torch.ones(N, N, dtype=torch.bool, device=q.device).triu(1), float("-inf"))
    lse = torch.logsumexp(s, -1)
    o = (torch.softmax(s, -1) @ vf).to(q.dtype)
    return o.transpose(1, 2).contiguous().transpose(1, 2), lse


@attn.register_fake
def _attn_fake(qkv, cos, sin, n_heads):
    B, N, three_d = qkv.shape
    dk = three_d // (3 * n_heads)
    o = qkv.new_empty((B, N, n_heads, dk)).permute(0, 2, 1, 3)
    return o, qkv.new_empty((B, n_heads, N), dtype=torch.float32)


@torch.library.custom_op("cs336c::attn_bwd", mutates_args=())
def attn_bwd(do: Tensor, qkv: Tensor, o: Tensor, lse: Tensor, cos: Tensor, sin: Tensor, n_heads: int) -> Tensor:
    """d(qkv) of :func:`attn` w.r.t. the UN-rotated q|k (the inverse RoPE applied to dQ/dK)."""
    q, k, v = _split(qkv, n_heads)
    B, N = qkv.shape[0], qkv.shape[1]
    dqkv = torch.empty_like(qkv)
    dq, dk_, dv = _split(dqkv, n_heads)
    if do.stride(-1) != 1:
        do = do.contiguous()
    if _hip_ok(qkv):
        scale = q.shape[-1] ** -0.5
        if N <= cos.shape[0]:
            _hip().fa_bwd_into(do, q, k, v, o, lse, True, scale, dq, dk_, dv, cos, sin, None, True)
        else:
            _hip().fa_bwd_into(do, q, k, v, o, lse, True, scale, dq, dk_, dv)
            dqk = dqkv.view(B, N, 3, n_heads, -1)[:, :, 0:2].reshape(B, N, 2 * n_heads, -1).transpose(1, 2)
            _hip().rope_into(dqk, cos, sin, None, True, dqk)
        return dqkv
    # reference backward in closed form (autograd does not record below a custom op)
    scale = q.shape[-1] ** -0.5
    qf, kf, vf, dof = q.float(), k.float(), v.float(), do.float()
    s = qf @ kf.transpose(-1, -2) * scale
    s = s.masked_fill(torch.ones(N, N, dtype=torch.bool, device=q.device).triu(1), float("-inf"))
    p = torch.softmax(s, -1)
    gv = p.transpose(-1, -2) @ dof
    dp = dof @ vf.transpose(-1, -2)
    ds = p * (dp - (dp * p).sum(-1, keepdim=True))
    gq, gk = ds @ kf * scale, ds.transpose(-1, -2) @ qf * scale
    pos = torch.arange(N, device=q.device)
    # inverse rotation of dQ / dK (rotation by -theta: cos, -sin)
    dq.copy_(rope_ref(gq, cos, -sin, pos).to(dq.dtype))
    dk_.copy_(rope_ref(gk, cos, -sin, pos).to(dk_.dtype))
    dv.copy_(gv.to(dv.dtype))
    return dqkv


@attn_bwd.register_fake
def _attn_bwd_fake(do, qkv, o, lse, cos, sin, n_heads):
    return torch.empty_like(qkv)


def _attn_setup(ctx, inputs, output):
    qkv, cos, sin, n_heads = inputs
    o, lse = output
    ctx.mark_non_differentiable(lse)
    ctx.save_for_backward(qkv, o, lse, cos, sin)
    ctx.n_heads = n_heads


def _attn_backward(ctx, do, _dlse):
    qkv, o, lse, cos, sin = ctx.saved_tensors
    return attn_bwd(do, qkv, o, lse, cos, sin, ctx.n_heads), None, None, None


attn.register_autograd(_attn_backward, setup_context=_attn_setup)


# ------------------------------------------------------------------------------------------
# SwiGLU feed-forward with the gate in the GEMM epilogues
# ------------------------------------------------------------------------------------------
@torch.library.custom_op("cs336c::swiglu_ffn", mutates_args=())
def _swiglu_ffn(x2: Tensor, w1: Tensor, w3: Tensor, w2: Tensor) -> Tuple[Tensor, Tensor, Tensor, Tensor, Tensor]:
    """(out, y = x2·[W1;W3]ᵀ, h = silu(y_a)·y_b, [W1;W3]ᵀ, W2ᵀ) in bf16; out = h·W2ᵀ. The two Wᵀ are
    the backward's K-major operands (saved, never re-cast there)."""
    x = _cast(x2, _BF16)
    w13, w13t = _weights([w1, w3], _BF16)
    w2b, w2t = _weights([w2], _BF16)
    if _hip_ok(x):
        half = w13.shape[0] // 2
        if gemm.gemm8_ok(x, w13, 1, half):
            y, h = gemm.gemm8_swiglu_fwd(x, w13)
        else:
            y = gemm.mm_nt(x, w13)
            h = _hip().swiglu_fused_fwd(y)
        return gemm.mm_nt(h, w2b), y, h, w13t, w2t
    y = x @ w13.t()
    a, b = y.float().chunk(2, -1)
    h = (a * torch.sigmoid(a) * b).to(_BF16)
    return h @ w2b.t(), y, h, w13t, w2t


@_swiglu_ffn.register_fake
def _swiglu_ffn_fake(x2, w1, w3, w2):
    T, d = x2.shape[0], w1.shape[1]
    return (x2.new_empty((T, w2.shape[0]), dtype=_BF16), x2.new_empty((T, 2 * w1.shape[0]), dtype=_BF16),
            x2.new_empty((T, w1.shape[0]), dtype=_BF16), x2.new_empty((d, 2 * w1.shape[0]), dtype=_BF16),
            x2.new_empty((w2.shape[1], w2.shape[0]), dtype=_BF16))


def swiglu_ffn(x2: Tensor, w1: Tensor, w3: Tensor, w2: Tensor) -> Tuple[Tensor, Tensor, Tensor]:
    out, y, h, _, _ = _swiglu_ffn(x2, w1, w3, w2)
    return out, y, h


@torch.library.custom_op("cs336c::swiglu_ffn_bwd", mutates_args=())
def swiglu_ffn_bwd(dout: Tensor, x2: Tensor, y: Tensor, h: Tensor, w13t: Tensor, w2t: Tensor,
                   need_dx: bool) -> Tuple[Tensor, Tensor, Tensor]:
    """(dX, fp32 dW13 = d[W1;W3], fp32 dW2) of :func:`swiglu_ffn`, from the forward's saved Wᵀ."""
    dy = _cast(dout, _BF16)
    x = _cast(x2, _BF16)
    half = y.shape[1] // 2
    if _hip_ok(dy):
        dw2 = gemm.mm_dw(dy, h) if gemm.dw_g8w_ok(dy, h) else gemm.mm_tn_fp32(dy, h)
        if gemm.gemm8_ok(dy, w2t, 2, half) and gemm._aligned_rows(y):
            dab = gemm.gemm8_swiglu_bwd(dy, w2t, y)
        else:
            dab = _hip().swiglu_fused_bwd(gemm.mm_nt(dy, w2t).contiguous(), y)
        dx = gemm.mm_nt(dab, w13t) if need_dx else dy.new_empty((0,))
        dw13 = gemm.mm_dw(dab, x) if gemm.dw_g8w_ok(dab, x) else gemm.mm_tn_fp32(dab, x)
        return dx, dw13, dw2
    dw2 = dy.t().float() @ h.float()
    dh = dy.float() @ w2t.float().t()
    a, b = y.float()[:, :half], y.float()[:, half:]
    s = torch.sigmoid(a)
    dab = torch.cat((dh * b * s * (1 + a * (1 - s)), dh * a * s), 1).to(_BF16)
    dx = (dab.float() @ w13t.float().t()).to(_BF16) if need_dx else dy.new_empty((0,))
    return dx, dab.t().float() @ x.float(), dw2


@swiglu_ffn_bwd.register_fake
def _swiglu_ffn_bwd_fake(dout, x2, y, h, w13t, w2t, need_dx):
    dx = x2.new_empty(x2.shape if need_dx else (0,), dtype=_BF16)
    return (dx, x2.new_empty((w13t.shape[1], x2.shape[1]), dtype=torch.float32),
            x2.new_empty((w2t.shape[1], w2t.shape[0]), dtype=torch.float32))


def _swiglu_setup(ctx, inputs, output):
    x2, w1, w3, w2 = inputs
    _, y, h, w13t, w2t = output
    ctx.mark_non_differentiable(y, h, w13t, w2t)
    ctx.save_for_backward(x2, y, h, w13t, w2t)
    ctx.x_dtype = x2.dtype
    ctx.rows1 = w1.shape[0]
    ctx.wdtypes = (w1.dtype, w3.dtype, w2.dtype)


def _swiglu_backward(ctx, dout, _dy, _dh, _dw13t, _dw2t):
    x2, y, h, w13t, w2t = ctx.saved_tensors
    need_dx = ctx.needs_input_grad[0]
    dx, dw13, dw2 = swiglu_ffn_bwd(dout, x2, y, h, w13t, w2t, need_dx)
    dw1, dw3 = dw13.split(ctx.rows1, 0)
    return ((_cast(dx, ctx.x_dtype) if need_dx else None), _cast(dw1, ctx.wdtypes[0]), _cast(dw3, ctx.wdtypes[1]),
            _cast(dw2, ctx.wdtypes[2]))


_swiglu_ffn.register_autograd(_swiglu_backward, setup_context=_swiglu_setup)


# ------------------------------------------------------------------------------------------
# token embedding with the deterministic HIP backward
# ------------------------------------------------------------------------------------------
@torch.library.custom_op("cs336c::embedding", mutates_args=())
def embedding(ids: Tensor, weight: Tensor) -> Tensor:
    """``weight[ids]``. Traced as an opaque op so that its backward is the HIP kernel of
    ``csrc/ops/embedding.hip`` (stable sort + one workgroup per vocabulary row, no atomics) instead of
    Inductor's decomposition of ``embedding_dense_backward`` (an index_put with float atomics:
    1.75 ms per 2.7b step at batch 4 against 0.03 ms, ``profiles/r6_compile.md``)."""
    return torch.nn.functional.embedding(ids, weight)


@embedding.register_fake
def _embedding_fake(ids, weight):
    return weight.new_empty((*ids.shape, weight.shape[1]))


@torch.library.custom_op("cs336c::embedding_bwd", mutates_args=())
def embedding_bwd(g: Tensor, ids: Tensor, vocab: int) -> Tensor:
    """fp32 (vocab, d) gradient of :func:`embedding`."""
    d = g.shape[-1]
    g2 = g.reshape(-1, d)
    if _hip_ok(g2) and d % 4 == 0:
        if not g2.is_contiguous():
            g2 = g2.contiguous()
        sorted_ids, perm = torch.sort(ids.reshape(-1), stable=True)
        return _hip().embedding_bwd(g2, sorted_ids, perm, vocab)
    gw = torch.zeros((vocab, d), dtype=torch.float32, device=g.device)
    return gw.index_add_(0, ids.reshape(-1), g2.float())


@embedding_bwd.register_fake
def _embedding_bwd_fake(g, ids, vocab):
    return g.new_empty((vocab, g.shape[-1]), dtype=torch.float32)


def _embedding_setup(ctx, inputs, output):
    ids, weight = inputs
    ctx.save_for_backward(ids)
    ctx.vocab, ctx.wdtype = weight.shape[0], weight.dtype


def _embedding_backward(ctx, g):
    (ids,) = ctx.saved_tensors
    return None, _cast(embedding_bwd(g, ids, ctx.vocab), ctx.wdtype)


embedding.register_autograd(_embedding_backward, setup_context=_embedding_setup)


# ------------------------------------------------------------------------------------------
# Inductor: explicit fallback lowerings for the opaque ops
# ------------------------------------------------------------------------------------------
def register_inductor_fallbacks(namespaces=("cs336c", "cs336")) -> int:
    """Give every op of ``namespaces`` an explicit Inductor fallback lowering. Without one, Inductor
    creates an "implicit fallback" the first time it meets the op and formats its arguments for a
    log line before the log level is checked (``torch/_inductor/graph.py``, ``call_function``): the
    string of an IR node prints its whole input DAG as a tree, which is exponential in the depth of
    the backward graph -- the first ``rmsnorm_bwd`` of a 12-layer model's backward (layer 0's norm,
    every other layer's gradient path upstream of it) never finished formatting in 10 minutes.
    Returns the number of ops registered."""
    try:
        from torch._inductor.lowering import lowerings, make_fallback
    except Exception:  # noqa: BLE001 - Inductor internals moved: compile still works, only slower
        return 0
    n = 0
    all_ops = torch._C._dispatch_get_all_op_names()  # "ns::name" or "ns::name.overload"
    for ns_name in namespaces:
        names = sorted({o.split("::", 1)[1].split(".")[0] for o in all_ops if o.startswith(ns_name + "::")})
        for name in names:
            try:
                packet = getattr(getattr(torch.ops, ns_name), name)
                if not isinstance(packet, torch._ops.OpOverloadPacket):
                    continue
                for ov in packet.overloads():
                    op = getattr(packet, ov)
                    if op not in lowerings:
                        make_fallback(op, warn=False)
                        n += 1
            except Exception:  # noqa: BLE001 - never let this break loading the ops
                continue
    return n


register_inductor_fallbacks(("cs336c",))
