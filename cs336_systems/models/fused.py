"""Fused weight layout and mixed-precision GEMM path for MI355X.

Three ideas, all invisible to the state dict (parameter names/shapes are the reference's):

1. **Grouped parameters.** ``q_proj/k_proj/v_proj`` and ``w1/w3`` keep their own ``nn.Parameter``
   objects, but their storage is re-allocated as consecutive row blocks of ONE tensor
   (:func:`group_params_`). The forward then runs a single GEMM per group (N = 3·d_model for QKV,
   2·d_ff for W1|W3) instead of three/two narrow ones — the d×d projections are the least
   efficient hipBLASLt shapes of the model (their dW has only ~40 output tiles for 256 CUs).
2. **bf16 compute-weight shadows.** A bf16 copy of every weight, laid out like the fp32 masters
   (groups stay contiguous), is written by the fused AdamW kernel in the same pass as the update
   (+2 B/param) instead of autocast re-casting all 2 B fp32 weights every forward (6 B/param in
   separate kernels). Shadows are used only while ``p._version`` matches the version recorded when
   they were written, so any out-of-band change of a master weight falls back to casting.
3. **fp32 weight gradients straight from the GEMM.** ``dW = dYᵀ X`` is computed by hipBLASLt with
   bf16 inputs and an fp32 output (``aten::mm.dtype``), so there is no bf16→fp32 cast kernel per
   weight in backward.

:class:`AttentionCore` and :class:`SwiGLUGate` consume the fused projection outputs in place
(strided views: no split/cat copies) and produce the fused dY for the grouped GEMM's backward.
"""

from __future__ import annotations

import os

import torch
import torch.nn as nn

from .. import ops
from ..ops import gemm
from ..ops._ext import ops as _hip

_SHADOW = "_cs336_bf16"
_SHADOW_VER = "_cs336_bf16_ver"
_SHADOW_GEN = "_cs336_bf16_gen"  # bumped on every shadow (re)write
_SHADOW_T = "_cs336_bf16t"  # transposed bf16 shadow Wᵀ (d_in, d_out) view, written by the fused AdamW
_SHADOW_T_GEN = "_cs336_bf16t_gen"  # shadow generation the Wᵀ was written at


# ------------------------------------------------------------------------------------------
# grouped storage
# ------------------------------------------------------------------------------------------
_GROUP_SEQ = 0


@torch.no_grad()
def group_params_(params: list[nn.Parameter]) -> torch.Tensor:
    """Re-home ``params`` (2-D, same width/dtype/device) as consecutive row blocks of one tensor."""
    global _GROUP_SEQ
    _GROUP_SEQ += 1
    gid = _GROUP_SEQ
    d_in = params[0].shape[1]
    rows = sum(p.shape[0] for p in params)
    base = torch.empty(rows, d_in, dtype=params[0].dtype, device=params[0].device)
    off = 0
    for p in params:
        n = p.shape[0]
        base[off : off + n].copy_(p.data)
        p.data = base[off : off + n]
        off += n
        # group tag: DDP bucketing keeps a group together even after another wrapper (ZeRO-1's flat
        # buffers) has moved every parameter into one storage
        p._cs336_group = gid
    return base


def _adjacent_rows(ts: list[torch.Tensor]) -> torch.Tensor | None:
    """If ``ts`` are row-adjacent contiguous blocks of one storage, return the combined 2-D view."""
    t0 = ts[0]
    if t0.dim() != 2 or not t0.is_contiguous():
        return None
    d_in = t0.shape[1]
    ptr = t0.untyped_storage().data_ptr()
    off = t0.storage_offset()
    rows = 0
    for t in ts:
        if (
            t.dim() != 2
            or t.shape[1] != d_in
            or not t.is_contiguous()
            or t.dtype != t0.dtype
            or t.untyped_storage().data_ptr() != ptr
            or t.storage_offset() != off + rows * d_in
        ):
            return None
        rows += t.shape[0]
    return torch.as_strided(t0.detach(), (rows, d_in), (d_in, 1), off)


def grouped_view(params: list[nn.Parameter]) -> torch.Tensor | None:
    return _adjacent_rows(list(params))


# ------------------------------------------------------------------------------------------
# bf16 shadows
# ------------------------------------------------------------------------------------------
def has_shadow(p: torch.Tensor) -> bool:
    return getattr(p, _SHADOW, None) is not None


def shadow_valid(p: torch.Tensor) -> bool:
    return getattr(p, _SHADOW, None) is not None and getattr(p, _SHADOW_VER, None) == p._version


def get_shadow(p: torch.Tensor) -> torch.Tensor | None:
    return getattr(p, _SHADOW, None)


def mark_shadow_synced(p: torch.Tensor) -> None:
    setattr(p, _SHADOW_VER, p._version)
    setattr(p, _SHADOW_GEN, getattr(p, _SHADOW_GEN, 0) + 1)


def get_shadow_t(p: torch.Tensor) -> torch.Tensor | None:
    return getattr(p, _SHADOW_T, None)


def mark_shadow_t_synced(p: torch.Tensor) -> None:
    """Wᵀ holds the transpose of the CURRENT shadow (call right after mark_shadow_synced)."""
    setattr(p, _SHADOW_T_GEN, getattr(p, _SHADOW_GEN, 0))


def shadow_t_valid(p: torch.Tensor) -> bool:
    """Wᵀ is usable iff the shadow is valid and Wᵀ was written with that very shadow generation
    (any other shadow refresh -- a cast after a ZeRO gather, say -- bumps the generation)."""
    return (
        getattr(p, _SHADOW_T, None) is not None
        and shadow_valid(p)
        and getattr(p, _SHADOW_T_GEN, -1) == getattr(p, _SHADOW_GEN, 0)
    )


@torch.no_grad()
def attach_bf16_shadows(module_or_params, transposed: bool | None = None) -> int:
    """Allocate bf16 shadows for every 2-D fp32 GPU weight (grouped weights get one contiguous
    shadow per group, mirroring the master layout) and fill them. Returns #params.

    ``transposed`` (default: ``CS336_WT`` != 0) also allocates Wᵀ shadows: each maximal run of
    row-adjacent, equally wide weights of one storage (a fused QKV or W1|W3 group, or neighbours in
    a ZeRO flat buffer) gets one (d_in, rows) bf16 tensor and every weight a column-block view of it,
    so a group's Wᵀ is again one strided view. The fused AdamW rewrites them with the update
    (``ops/adamw.py``), replacing the per-forward transpose of every weight."""
    src = module_or_params.parameters() if isinstance(module_or_params, nn.Module) else module_or_params
    params = [p for p in src if p.dim() == 2 and p.dtype == torch.float32 and p.is_cuda and not has_shadow(p)]
    if transposed is None:
        transposed = _transpose_weight()
    by_storage: dict[int, list[nn.Parameter]] = {}
    for p in params:
        by_storage.setdefault(p.untyped_storage().data_ptr(), []).append(p)
    for group in by_storage.values():
        group.sort(key=lambda t: t.storage_offset())
        base = group[0]
        st_numel = base.untyped_storage().nbytes() // base.element_size()
        shadow_base = torch.empty(st_numel, dtype=torch.bfloat16, device=base.device)
        for p in group:
            setattr(p, _SHADOW, torch.as_strided(shadow_base, p.shape, p.stride(), p.storage_offset()))
        if transposed:
            _attach_transposed(group)
    refresh_bf16_shadows(params, transposed=True)
    return len(params)


def _attach_transposed(group: list[nn.Parameter]) -> None:
    """Wᵀ views for ``group`` (one storage, sorted by offset): one (d_in, rows) tensor per run."""
    runs: list[list[nn.Parameter]] = []
    for p in group:
        if not p.is_contiguous() or p.shape[0] % 8 or p.shape[1] % 8:
            continue
        prev = runs[-1][-1] if runs else None
        if prev is not None and prev.shape[1] == p.shape[1] and p.storage_offset() == prev.storage_offset() + prev.numel():
            runs[-1].append(p)
        else:
            runs.append([p])
    for run in runs:
        d_in, rows = run[0].shape[1], sum(p.shape[0] for p in run)
        wt = torch.empty(d_in, rows, dtype=torch.bfloat16, device=run[0].device)
        off = 0
        for p in run:
            setattr(p, _SHADOW_T, wt[:, off : off + p.shape[0]])
            off += p.shape[0]


@torch.no_grad()
def refresh_bf16_shadows(params, transposed: bool = False) -> None:
    """Re-cast the shadows of ``params`` from their fp32 masters (one multi-tensor launch); with
    ``transposed`` also re-write their Wᵀ shadows (one transpose per weight: attach time only --
    elsewhere a stale Wᵀ just makes the forward transpose the weight itself)."""
    ps = [p for p in params if has_shadow(p)]
    if not ps:
        return
    if ops.ext_available() and all(p.is_contiguous() for p in ps):
        _hip().multi_tensor_cast_bf16([p.data for p in ps], [get_shadow(p) for p in ps])
    else:
        for p in ps:
            get_shadow(p).copy_(p.data)
    for p in ps:
        mark_shadow_synced(p)
        wt = get_shadow_t(p) if transposed else None
        if wt is not None:
            wt.copy_(get_shadow(p).t())
            mark_shadow_t_synced(p)


@torch.no_grad()
def refresh_transposed(params) -> int:
    """Re-write the Wᵀ shadows of ``params`` from their current bf16 shadows -- one transpose per run
    of row-adjacent weights that share one Wᵀ tensor (a fused QKV / W1|W3 group is one launch) --
    and mark them in sync. For weights whose shadow was refreshed outside the fused AdamW (ZeRO
    parameter gathers), so the next forward finds a valid Wᵀ instead of transposing each weight.
    Returns the number of transposes launched."""
    runs: dict[tuple, list] = {}
    for p in params:
        wt = get_shadow_t(p)
        if wt is None or not shadow_valid(p):
            continue
        runs.setdefault((wt.untyped_storage().data_ptr(), wt.shape[0]), []).append(p)
    n = 0
    for ps in runs.values():
        ps.sort(key=lambda t: get_shadow_t(t).storage_offset())
        src = _adjacent_rows([get_shadow(p) for p in ps])
        dst = _adjacent_cols([get_shadow_t(p) for p in ps])
        if src is not None and dst is not None and src.is_cuda and ops.ext_available() and src.shape[0] % 8 == 0:
            _hip().transpose2d_into(src, dst)
            n += 1
        else:
            for p in ps:
                s, st = get_shadow(p), get_shadow_t(p)
                ok = (s.is_cuda and s.dim() == 2 and st.dim() == 2 and s.stride(1) == 1 and st.stride(1) == 1
                      and s.shape[0] % 8 == 0 and s.shape[1] % 8 == 0 and s.stride(0) % 8 == 0 and st.stride(0) % 8 == 0
                      and s.data_ptr() % 16 == 0 and st.data_ptr() % 16 == 0 and ops.ext_available())
                if ok:
                    _hip().transpose2d_into(s, st)  # the HIP transpose, not a strided copy
                else:
                    st.copy_(s.t())
                n += 1
        for p in ps:
            mark_shadow_t_synced(p)
    return n


def _adjacent_cols(ts: list[torch.Tensor]) -> torch.Tensor | None:
    """If ``ts`` are column-adjacent blocks (unit column stride) of one storage, the combined view."""
    t0 = ts[0]
    if t0.dim() != 2 or t0.stride(1) != 1:
        return None
    ld, off, cols = t0.stride(0), t0.storage_offset(), 0
    ptr = t0.untyped_storage().data_ptr()
    for t in ts:
        if (
            t.dim() != 2
            or t.shape[0] != t0.shape[0]
            or t.stride() != (ld, 1)
            or t.untyped_storage().data_ptr() != ptr
            or t.storage_offset() != off + cols
        ):
            return None
        cols += t.shape[1]
    return torch.as_strided(t0, (t0.shape[0], cols), (ld, 1), off)


def compute_weight_t(params: list[nn.Parameter]) -> torch.Tensor | None:
    """The (d_in, rows) bf16 Wᵀ of a group (or single) of params from their transposed shadows,
    or None when any is missing/stale (the caller transposes the compute weight instead)."""
    if not all(shadow_t_valid(p) for p in params):
        return None
    return _adjacent_cols([get_shadow_t(p) for p in params])


def compute_weight(params: list[nn.Parameter], dtype: torch.dtype) -> torch.Tensor:
    """The (rows, d_in) weight in ``dtype`` for a group (or single) of params: the shadow view when
    valid, else one cast of the (grouped) master view, else a concatenation (ungrouped fallback)."""
    if dtype == torch.bfloat16 and all(shadow_valid(p) for p in params):
        v = _adjacent_rows([get_shadow(p) for p in params])
        if v is not None:
            return v
    g = grouped_view(params) if len(params) > 1 else params[0].detach()
    if g is None:
        g = torch.cat([p.detach() for p in params], 0)
    return g if g.dtype == dtype else g.to(dtype)


# ------------------------------------------------------------------------------------------
# weight-gradient side stream
# ------------------------------------------------------------------------------------------
# dW = dYᵀX is off backward's critical path (nothing in backward consumes it), so it CAN run on a
# second HIP stream while the main stream continues with dX and the memory-bound kernels of the
# next layers (RMSNorm/SwiGLU/RoPE backward, FA backward). The main stream waits for the side
# stream only where a weight gradient is consumed: before a DDP bucket / per-parameter all-reduce
# (sync_dw_stream) and at the end of the backward pass (an engine callback).
#
# OFF by default (CS336_DW_STREAM=1 enables it). Measured on MI355X: it saves only ~2 ms of a
# ~187 ms XL step, because the hipBLASLt GEMMs hold ~1 workgroup per CU and the HBM-bound kernels
# next to them run 3-5x slower (profiles/r1_overlap_ab.json).
#
# Concurrent GEMMs and the round-1 hang: hipBLASLt's default picks for every projection GEMM are
# stream-K Tensile kernels (SK3): a grid of <= 1 workgroup per CU in which the owner of a split tile
# spins on a workspace flag written by the next-indexed workgroup (profiles/r2_streamk_hang.md). Two
# of them on two streams need more slots than the chip has, each kernel's resident workgroups wait for
# undispatched successors, and neither finishes -- the 2.7b step hung exactly so with the dW GEMMs on
# this stream. hipBLASLt has no data-parallel alternative for these problems on gfx950 (2198 of
# its 2199 solutions are stream-K, scripts/lt_dp_probe.py), so a weight gradient goes to the side
# stream only if the cs336 MFMA GEMM (whole tiles per workgroup, no inter-workgroup waits) takes it
# (gemm.dw_concurrent_ok); otherwise it runs on the main stream. A cs336 GEMM beside an RCCL
# kernel only waits for it (tests/test_concurrency_gpu.py); a stream-K grid beside RCCL is the
# hazard cs336_systems/rccl_env.py caps (profiles/r3_coresidency.md).
_SIDE_STREAMS: dict[int, torch.cuda.Stream] = {}
_state = {"dirty": False, "callback": False}
# Inputs of in-flight side-stream dW GEMMs, oldest first: (event recorded after the GEMM, the
# main-stream tensors it reads). They are held here instead of ``record_stream``-ed: a block
# freed with a side-stream use cannot be reused until the allocator sees that use complete, and
# with the host steps ahead of the GPU every layer's dY / X then needs a fresh block
# (profiles/r4_dw_stream.md). Past _SIDE_LAG entries the main stream waits for the oldest GEMM
# and the tensors are released in main-stream order.
_SIDE_PENDING: list[tuple[torch.cuda.Event, tuple[torch.Tensor, ...]]] = []
_SIDE_LAG = 2


def _hold_for_side(main: torch.cuda.Stream, side: torch.cuda.Stream, *ts: torch.Tensor) -> None:
    ev = torch.cuda.Event()
    ev.record(side)
    _SIDE_PENDING.append((ev, ts))
    while len(_SIDE_PENDING) > _SIDE_LAG:
        old, _ = _SIDE_PENDING.pop(0)
        main.wait_event(old)


def dw_stream_enabled() -> bool:
    return os.environ.get("CS336_DW_STREAM", "0") == "1"


def _side_stream(device: torch.device) -> torch.cuda.Stream:
    idx = device.index if device.index is not None else torch.cuda.current_device()
    s = _SIDE_STREAMS.get(idx)
    if s is None:
        s = _SIDE_STREAMS[idx] = torch.cuda.Stream(device=idx)
    return s


def sync_dw_stream() -> None:
    """Make the current stream wait for every weight-gradient GEMM issued so far."""
    if not _state["dirty"]:
        return
    _state["dirty"] = False
    for idx, s in _SIDE_STREAMS.items():
        torch.cuda.current_stream(idx).wait_stream(s)
    _SIDE_PENDING.clear()  # after the wait: their blocks are reused in main-stream order


def dw_stream_for(t: torch.Tensor) -> torch.cuda.Stream | None:
    """The side stream of ``t``'s device if weight-gradient work is pending on it, else None."""
    if not (_state["dirty"] and t.is_cuda):
        return None
    return _SIDE_STREAMS.get(t.device.index if t.device.index is not None else torch.cuda.current_device())


def _end_of_backward() -> None:
    _state["callback"] = False
    sync_dw_stream()


def _save_transposed(k_in: int, n_out: int) -> bool:
    """Save Xᵀ for the weight gradient when N_out / K_in >= CS336_XT_RATIO (default 4; 0 = off).
    Measured per XL projection: W1|W3 (ratio 8) gains 0.19 ms/layer; QKV (3) and O (1) gain less
    than the transpose costs; W2 (0.25) loses."""
    r = float(os.environ.get("CS336_XT_RATIO", "4"))
    return r > 0 and n_out >= r * k_in


def _transpose(t: torch.Tensor) -> torch.Tensor:
    """``t.t().contiguous()`` via the tiled HIP transpose (csrc/ops/transpose.hip) when it applies."""
    if (
        t.is_cuda
        and t.dim() == 2
        and t.element_size() == 2
        and t.stride(1) == 1
        and t.shape[0] % 8 == 0
        and t.shape[1] % 8 == 0
        and t.stride(0) % 8 == 0
        and t.data_ptr() % 16 == 0
        and ops.ext_available()
    ):
        return _hip().transpose2d(t)
    return t.t().contiguous()


def _transpose_weight() -> bool:
    return os.environ.get("CS336_WT", "1") != "0"


def _dy_transposed(k_in: int, n_out: int) -> bool:
    """Transpose dY for the weight gradient of narrow projections (N_out <= K_in: the attention
    output projection and W2, whose dY is the residual-stream gradient). dYᵀ·X (or dYᵀ·(Xᵀ)ᵀ with Oᵀ)
    reads the token dimension contiguously on the dY side, which hipBLASLt runs 1.2x (W2) to 1.4x
    (O with Oᵀ) faster than dY token-major (profiles/r2_gemm_ab_epi.json), for one transpose of a
    (tokens, N_out) bf16 tensor. CS336_DYT=0: off."""
    return os.environ.get("CS336_DYT", "1") != "0" and n_out <= k_in


# Transposed bf16 gradients written by their producer (the fused residual RMSNorm backward) for
# the weight-gradient GEMM of the projection that consumes the row-major copy: keyed by the row-major
# tensor's data pointer; the entry holds that tensor, so its storage (and address) cannot be reused
# while the entry lives. At most a few entries (an unconsumed offer is dropped oldest-first).
_DYT_OFFERS: "dict[int, tuple[torch.Tensor, torch.Tensor]]" = {}


def offer_transposed_grad(g: torch.Tensor, gt: torch.Tensor) -> None:
    _DYT_OFFERS[g.data_ptr()] = (g, gt)
    while len(_DYT_OFFERS) > 4:
        _DYT_OFFERS.pop(next(iter(_DYT_OFFERS)))


def take_transposed_grad(g2: torch.Tensor) -> torch.Tensor | None:
    """The producer-written ``g2ᵀ`` for a 2-D row-major gradient ``g2`` (same storage, same
    element count, same dtype), or None."""
    e = _DYT_OFFERS.pop(g2.data_ptr(), None)
    if e is None:
        return None
    g, gt = e
    ok = (g.numel() == g2.numel() and g.dtype == g2.dtype and g2.is_contiguous()
          and gt.shape == (g2.shape[1], g2.shape[0]) and gt.dtype == g2.dtype)
    return gt if ok else None


def _rope_out_in_fa() -> bool:
    """Fuse the backward's inverse RoPE into the FA2 backward's dQ/dK store (CS336_FA_ROPE_OUT=0: off)."""
    return os.environ.get("CS336_FA_ROPE_OUT", "1") != "0"


def attn_out_transposed() -> bool:
    """The FA2 forward also writes Oᵀ for the output projection's weight gradient (CS336_OT=1: on).
    Off by default: with dYᵀ for that GEMM the O-side layout gains less than the forward's extra
    transposed store costs (same-box A/B on XL: 180.8 ms/step off vs 181.0 on)."""
    return os.environ.get("CS336_OT", "0") == "1"


def _mark_side_work() -> None:
    _state["dirty"] = True
    if not _state["callback"]:
        _state["callback"] = True
        torch.autograd.Variable._execution_engine.queue_callback(_end_of_backward)


# ------------------------------------------------------------------------------------------
# fused linear
# ------------------------------------------------------------------------------------------
def _mm_fp32_out(a: torch.Tensor, b: torch.Tensor) -> torch.Tensor:
    """a @ b with an fp32 result: bf16 x bf16 -> fp32 in one hipBLASLt call when available."""
    if a.dtype == torch.bfloat16 and a.is_cuda:
        try:
            return torch.mm(a, b, out_dtype=torch.float32)
        except (TypeError, RuntimeError):
            pass
    return torch.mm(a, b).float()


class FusedLinearFn(torch.autograd.Function):
    """y = x @ [W_0; W_1; ...]^T for a group of weights with one GEMM; grads come back as row
    views of one fp32 dW."""

    @staticmethod
    def forward(ctx, x, xt_given, *weights):
        amp = torch.is_autocast_enabled("cuda") and x.is_cuda
        cdt = torch.get_autocast_dtype("cuda") if amp else weights[0].dtype
        w = compute_weight(list(weights), cdt)
        x2 = x.reshape(-1, x.shape[-1])
        if x2.dtype != cdt:
            x2 = x2.to(cdt)
        # (a fused consumer -- SwiGLUFFNFn -- may supply its own GEMM with an epilogue)
        mm = getattr(ctx, "mm_override", None) or gemm.mm_nt
        y = mm(x2, w)
        # For wide projections (N_out >= r * K_in, e.g. W1|W3: 12800 vs 1600) save Xᵀ instead of X:
        # the weight-gradient GEMM dYᵀX then reads both operands token-contiguous, which hipBLASLt
        # runs 1.4x faster on MI355X (profiles/r1_gemm_dw_layouts.json), for one small transpose.
        # A producer may hand over Xᵀ it wrote anyway (``xt_given``: the attention output's Oᵀ,
        # written by the FA2 forward), which makes the token-contiguous dW free for that projection.
        use_given = (
            xt_given is not None
            and xt_given.dtype == cdt
            and xt_given.shape == (x2.shape[1], x2.shape[0])
            and xt_given.stride(1) == 1
        )
        # weight gradient by gemm8w straight from token-major X and dY: save X as is, no Xᵀ / dYᵀ
        ctx.dw_g8w = (any(ctx.needs_input_grad[1:]) and x2.is_cuda and x2.dtype == torch.bfloat16
                      and gemm.dw_g8w_enabled() and gemm._aligned_rows(x2) and x2.shape[0] % 64 == 0
                      and gemm._dw_plan(x2.shape[0], w.shape[0], x2.shape[1]) is not None)
        ctx.xt = x2.is_cuda and any(ctx.needs_input_grad[1:]) and not ctx.dw_g8w and (
            use_given or _save_transposed(x2.shape[1], w.shape[0]))
        # The input-gradient GEMM dY·W reads W k-strided; from a transposed copy Wᵀ both operands
        # are K-major, which hipBLASLt runs 1.15-1.4x faster (profiles/r1_gemm_dw_layouts.json).
        # Wᵀ is made on the side stream right here, off the forward's critical path.
        ctx.wt_event = None
        ctx.w_t = x2.is_cuda and ctx.needs_input_grad[0] and w.dtype == torch.bfloat16 and _transpose_weight()
        wt_shadow = compute_weight_t(list(weights)) if ctx.w_t else None
        if wt_shadow is not None:  # Wᵀ written by the fused AdamW together with the bf16 shadow
            w_saved = wt_shadow
        elif ctx.w_t and (torch.cuda.is_current_stream_capturing() or torch.compiler.is_compiling()):
            # inside a HIP-graph capture or a torch.compile trace: stay on the current stream (no
            # side-stream events in a captured/traced region)
            w_saved = _transpose(w)
        elif ctx.w_t:
            main = torch.cuda.current_stream(x2.device)
            s = _side_stream(x2.device)
            s.wait_stream(main)
            with torch.cuda.stream(s):
                w_saved = _transpose(w)
            w.record_stream(s)
            ctx.wt_event = torch.cuda.Event()
            ctx.wt_event.record(s)
        else:
            w_saved = w
        if ctx.xt:
            x_saved = xt_given if use_given else _transpose(x2)
        else:
            x_saved = x2
        ctx.save_for_backward(x_saved, w_saved)
        ctx.x_shape = x.shape
        ctx.x_dtype = x.dtype
        ctx.rows = [p.shape[0] for p in weights]
        ctx.wdtype = [p.dtype for p in weights]
        ctx.weights = weights
        return y.view(*x.shape[:-1], y.shape[-1])

    @staticmethod
    def _grad_target(weights) -> torch.Tensor | None:
        """A DDP bucket region to write dW into (all grads unset, fp32, row-adjacent views)."""
        outs = [getattr(p, "_cs336_grad_out", None) for p in weights]
        if any(o is None for o in outs) or any(p.grad is not None for p in weights):
            return None
        if outs[0].dtype != torch.float32:
            return None
        return _adjacent_rows(outs)

    @staticmethod
    def backward(ctx, dy):
        x2, w = ctx.saved_tensors
        dy2 = dy.reshape(-1, dy.shape[-1])
        if dy2.dtype != w.dtype:
            dy2 = dy2.to(w.dtype)
        dx = dw_parts = None
        if ctx.needs_input_grad[0] and not getattr(ctx, "skip_dx", False):
            if ctx.w_t:  # w holds Wᵀ (K_in, N_out), made on the side stream (or in-stream under capture)
                if ctx.wt_event is not None:
                    main = torch.cuda.current_stream(dy2.device)
                    main.wait_event(ctx.wt_event)
                    w.record_stream(main)
                dx = gemm.mm_nt(dy2, w).view(ctx.x_shape)
            else:
                dx = gemm.mm_nn(dy2, w).view(ctx.x_shape)
            if dx.dtype != ctx.x_dtype:
                dx = dx.to(ctx.x_dtype)
        if any(ctx.needs_input_grad[1:]):
            target = FusedLinearFn._grad_target(ctx.weights) if dy2.dtype == torch.bfloat16 else None
            g8w = getattr(ctx, "dw_g8w", False) and gemm.dw_g8w_ok(dy2, x2)
            # side stream only when the grads are unset: AccumulateGrad then adopts dW without a
            # kernel (an accumulate-add on the main stream would race the side-stream GEMM); and only
            # for a data-parallel cs336 kernel (gemm8w, or the cs336 GEMM): never a stream-K GEMM
            # beside another GEMM
            side = (
                dy2.is_cuda
                and dy2.dtype == torch.bfloat16
                and not torch.is_grad_enabled()
                and dw_stream_enabled()
                and all(p.grad is None for p in ctx.weights)
                and all(dt == torch.float32 for dt in ctx.wdtype)
                and (g8w or gemm.dw_concurrent_ok(dy2, x2, ctx.xt))
            )
            dyt = None
            if g8w:
                take_transposed_grad(dy2)  # drop a producer's dYᵀ offer: not needed
            elif not side and dy2.is_cuda and dy2.dtype == torch.bfloat16 and _dy_transposed(ctx.x_shape[-1], dy2.shape[1]):
                dyt = take_transposed_grad(dy2)
                if dyt is None:
                    dyt = _transpose(dy2)
            if g8w:  # token-major dY and X, fp32 dW (straight into the DDP bucket when there is one)
                dw_fn = lambda out=None, cs=False: gemm.mm_dw(dy2, x2, out=out)  # noqa: E731
            elif dyt is not None:  # dYᵀ (N_out, tokens); x2 is X or Xᵀ
                dw_fn = lambda out=None, cs=False: gemm.mm_dyt_fp32(dyt, x2, ctx.xt, out=out)  # noqa: E731
            elif ctx.xt:  # x2 holds Xᵀ (K_in, tokens)
                dw_fn = lambda out=None, cs=False: gemm.mm_tn_fp32_xt(dy2, x2, out=out, concurrent_safe=cs)  # noqa: E731
            else:
                dw_fn = lambda out=None, cs=False: gemm.mm_tn_fp32(dy2, x2, out=out, concurrent_safe=cs)  # noqa: E731
            if side:
                main = torch.cuda.current_stream(dy2.device)
                s = _side_stream(dy2.device)
                s.wait_stream(main)
                with torch.cuda.stream(s):
                    dw = dw_fn(target, True)  # beside the main stream's GEMMs: no stream-K
                _hold_for_side(main, s, dy2, x2)
                if target is None:
                    dw.record_stream(main)
                _mark_side_work()
            elif target is not None or (dy2.dtype == torch.bfloat16 and dy2.is_cuda):
                dw = dw_fn(target)
            else:
                dw = _mm_fp32_out(dy2.t(), x2.t() if ctx.xt else x2)
            dw_parts = list(torch.split(dw, ctx.rows, 0))
            dw_parts = [g if g.dtype == dt else g.to(dt) for g, dt in zip(dw_parts, ctx.wdtype)]
        return (dx, None, *(dw_parts if dw_parts is not None else [None] * len(ctx.rows)))


def fused_linear(x: torch.Tensor, *weights: nn.Parameter, xt: torch.Tensor | None = None) -> torch.Tensor:
    """``x @ [W_0; W_1; ...]^T`` with one GEMM; ``xt`` optionally supplies ``x``'s (K_in, tokens)
    transpose for the weight gradient (see FusedLinearFn.forward)."""
    return FusedLinearFn.apply(x, xt, *weights)


# ------------------------------------------------------------------------------------------
# attention core on the fused QKV layout
# ------------------------------------------------------------------------------------------
class AttentionCore(torch.autograd.Function):
    """qkv (B, N, 3*H*dk) -> RoPE(q|k) -> causal FA2 -> o as a (B, H, N, dk) view of
    (B, N, H, dk) memory.

    Q and K heads are adjacent in the fused projection output, so one RoPE launch rotates both as
    a (B, 2H, N, dk) view. The backward writes dq, dk, dv straight into the three slices of one
    fused d(qkv) buffer, then one in-place inverse rotation covers dq|dk. No split/cat copies.

    (The FA kernels can also rotate Q/K on load — ``fa_fwd(..., cos, sin, pos)`` — but at
    N=512 that re-rotates every K tile once per query block and measured ~5 % slower per XL step
    than this one O(N) pass; see profiles/README.md.)"""

    @staticmethod
    def _split(t, H):
        B, N, three_d = t.shape
        dk = three_d // (3 * H)
        t5 = t.view(B, N, 3, H, dk)
        qk = t5[:, :, 0:2].reshape(B, N, 2 * H, dk).transpose(1, 2)  # view: (B, 2H, N, dk)
        return qk, t5[:, :, 2].transpose(1, 2)

    @staticmethod
    def forward(ctx, qkv, cos, sin, pos, H, want_ot=False, prerotated=False):
        # prerotated: the QKV GEMM applied RoPE to q|k in its store (QKVRopeLinearFn); the gradient
        # this backward returns is still w.r.t. the un-rotated projection output
        qk_in, v = AttentionCore._split(qkv, H)
        hip = _hip()
        qk = qk_in if prerotated else hip.rope(qk_in, cos, sin, pos, False)
        q, k = qk[:, :H], qk[:, H:]
        scale = q.shape[-1] ** -0.5
        if want_ot:  # also Oᵀ (H*dk, B*N), the output projection's token-contiguous dW operand
            o, lse, ot = hip.fa_fwd_ot(q, k, v, True, scale)
            ctx.mark_non_differentiable(ot)
        else:
            o, lse = hip.fa_fwd(q, k, v, True, scale)
            ot = None
        ctx.save_for_backward(qk, v, o, lse, cos, sin, pos)
        ctx.H, ctx.scale = H, scale
        return o, ot

    @staticmethod
    def backward(ctx, do, _dot=None):
        qk, v, o, lse, cos, sin, pos = ctx.saved_tensors
        H = ctx.H
        B, N = v.shape[0], v.shape[2]
        dqkv = torch.empty(B, N, 3 * H * v.shape[3], dtype=v.dtype, device=v.device)
        dqk, dv = AttentionCore._split(dqkv, H)
        if do.stride(-1) != 1:
            do = do.contiguous()
        hip = _hip()
        rpos = pos
        if rpos is not None and rpos.numel() != B * N:
            rpos = rpos.expand(B, N)
        if rpos is not None:
            rpos = rpos.contiguous()
        if _rope_out_in_fa() and N <= cos.shape[0]:
            # dQ/dK rotated back inside the FA2 backward's store (q/k were rotated by the forward's
            # RoPE pass): no separate inverse-RoPE pass over d(q|k)
            hip.fa_bwd_into(do, qk[:, :H], qk[:, H:], v, o, lse, True, ctx.scale, dqk[:, :H], dqk[:, H:], dv,
                            cos, sin, rpos, True)
        else:
            hip.fa_bwd_into(do, qk[:, :H], qk[:, H:], v, o, lse, True, ctx.scale, dqk[:, :H], dqk[:, H:], dv)
            hip.rope_into(dqk, cos, sin, pos, True, dqk)
        return dqkv, None, None, None, None, None, None


class QKVRopeLinearFn(torch.autograd.Function):
    """The fused QKV projection with RoPE applied to its q|k columns inside the GEMM's store
    (``gemm8`` epi 3): removes the separate forward RoPE pass (read + write of q|k per layer).

    The output holds ROTATED q|k, but autograd treats it as the plain projection output: its only
    consumer is :class:`AttentionCore` with ``prerotated=True``, whose backward returns the gradient
    w.r.t. the un-rotated q|k (the FA2 backward rotates dQ/dK back in its store), which is what this
    backward (the plain linear backward of :class:`FusedLinearFn`) needs."""

    @staticmethod
    def forward(ctx, x, cos, sin, pos, n_heads, *weights):
        sub = _SubCtx((True, False, *[w.requires_grad for w in weights]))
        B, N, _ = x.shape
        dk = weights[0].shape[0] // n_heads

        def mm(x2, w):
            if dk <= 96 and gemm.gemm8_ok(x2, w, 3, 2 * n_heads * dk):
                return gemm.gemm8_rope(x2, w, cos, sin, pos, N, 2 * n_heads * dk, dk)
            y2 = gemm.mm_nt(x2, w)
            qk, _ = AttentionCore._split(y2.view(B, N, -1), n_heads)
            _hip().rope_into(qk, cos, sin, pos, False, qk)
            return y2

        sub.mm_override = mm
        y = FusedLinearFn.forward(sub, x, None, *weights)
        sub.mm_override = None  # forward-only; the stage lives on as ctx.sub
        ctx.sub = sub
        _stash_saved(ctx, sub)
        return y

    @staticmethod
    def backward(ctx, dy):
        _unstash_saved(ctx, ctx.sub)
        dx, _, *dws = FusedLinearFn.backward(ctx.sub, dy)
        ctx.sub._saved = ()
        return (dx, None, None, None, None, *dws)


class _SubCtx:
    """Stand-in for an autograd ctx, so FusedLinearFn's forward/backward run as one stage of a
    larger Function (SwiGLUFFNFn) and keep all their logic: bf16/Wᵀ shadows, Xᵀ / dYᵀ layouts,
    fp32 dW written straight into the DDP bucket. The outer Function hands the stage's tensors to
    its own ``ctx.save_for_backward`` (:func:`_stash_saved`), so they get autograd's version-counter
    check, ``saved_tensors_hooks`` (checkpointing / offload) and ``retain_graph`` semantics."""

    def __init__(self, needs_input_grad):
        self.needs_input_grad = tuple(needs_input_grad)
        self._saved = ()

    def save_for_backward(self, *ts):
        self._saved = ts

    @property
    def saved_tensors(self):
        return self._saved


def _stash_saved(ctx, *subs, extra: tuple = ()) -> None:
    """Save the stages' tensors (then ``extra``) through the outer ``ctx.save_for_backward``; the
    stages keep only their counts (plain attributes bypassed version checks and hooks)."""
    ctx.sub_counts = [len(sub._saved) for sub in subs]
    ctx.save_for_backward(*[t for sub in subs for t in sub._saved], *extra)
    for sub in subs:
        sub._saved = ()


def _unstash_saved(ctx, *subs) -> tuple:
    """Give each stage back its saved tensors (version-checked by ``ctx.saved_tensors``); returns
    the ``extra`` tensors."""
    ts = ctx.saved_tensors
    i = 0
    for sub, n in zip(subs, ctx.sub_counts):
        sub._saved = tuple(ts[i : i + n])
        i += n
    return tuple(ts[i:])


def swiglu_fused_enabled() -> bool:
    """SwiGLU gate inside the gemm8 epilogues (CS336_SWIGLU_FUSED=0: separate HIP SwiGLU kernels)."""
    return os.environ.get("CS336_SWIGLU_FUSED", "1") != "0"


class SwiGLUFFNFn(torch.autograd.Function):
    """``w2(silu(w1 x) * w3 x)`` on the grouped W1|W3 layout with the gate fused into the GEMMs
    (``model.py:389-397``; kernels in ``csrc/gemm/gemm8.hip``):

    * forward: ONE kernel writes y = x·[W1;W3]ᵀ (saved) and h = silu(a)·b; then h·W2ᵀ;
    * backward: dW2 = dYᵀ·h, then ONE kernel computes dh = dY·W2 in registers and writes
      [da|db] = [dh·b·silu'(a) | dh·silu(a)] from the saved y (dh never reaches memory); then the
      W1|W3 input and weight gradients from [da|db].

    Removes both SwiGLU elementwise passes (read 2·d_ff + write d_ff, and read 3·d_ff + write 2·d_ff
    activations per token). Shapes the kernel does not take fall back to GEMM + SwiGLU kernel inside
    the same Function."""

    @staticmethod
    def forward(ctx, x, w1, w3, w2):
        c13 = _SubCtx((True, False, w1.requires_grad, w3.requires_grad))
        box = {}

        def mm13(x2, w):
            half = w.shape[0] // 2
            if gemm.gemm8_ok(x2, w, 1, half):
                y2, box["h"] = gemm.gemm8_swiglu_fwd(x2, w)
            else:
                y2 = gemm.mm_nt(x2, w)
                box["h"] = _hip().swiglu_fused_fwd(y2)
            return y2

        c13.mm_override = mm13
        y = FusedLinearFn.forward(c13, x, None, w1, w3)
        h = box.pop("h").view(*x.shape[:-1], -1)
        # the override is forward-only: the stage outlives this call (ctx.c13, for backward) and its
        # closure must not keep h alive past the backward that frees the saved copy (+30 GB on XL)
        c13.mm_override = None
        c2 = _SubCtx((True, False, w2.requires_grad))
        out = FusedLinearFn.forward(c2, h, None, w2)
        ctx.c13, ctx.c2 = c13, c2
        _stash_saved(ctx, c13, c2, extra=(y,))
        return out

    @staticmethod
    def backward(ctx, dout):
        c13, c2 = ctx.c13, ctx.c2
        (y,) = _unstash_saved(ctx, c13, c2)
        c2.skip_dx = True  # W2 stage: weight gradient only; its input gradient is fused below
        _, _, dw2 = FusedLinearFn.backward(c2, dout)
        h2, w2s = c2.saved_tensors
        dy2 = dout.reshape(-1, dout.shape[-1])
        if dy2.dtype != w2s.dtype:
            dy2 = dy2.to(w2s.dtype)
        y2 = y.reshape(-1, y.shape[-1])
        half = y2.shape[1] // 2
        if c2.w_t and c2.wt_event is not None:
            main = torch.cuda.current_stream(dy2.device)
            main.wait_event(c2.wt_event)
            w2s.record_stream(main)
        if c2.w_t and gemm.gemm8_ok(dy2, w2s, 2, half) and gemm._aligned_rows(y2):
            dab = gemm.gemm8_swiglu_bwd(dy2, w2s, y2)
        else:
            dh = gemm.mm_nt(dy2, w2s) if c2.w_t else gemm.mm_nn(dy2, w2s)
            dab = _hip().swiglu_fused_bwd(dh.contiguous(), y2)
        dx, _, dw1, dw3 = FusedLinearFn.backward(c13, dab.view(*y.shape))
        # drop the stages' references now (autograd frees its SavedVariables after this backward
        # unless retain_graph; a stage reference would keep every layer's h / X alive: +18 GiB on XL)
        c13._saved = c2._saved = ()
        return dx, dw1, dw3, dw2


class SwiGLUGate(torch.autograd.Function):
    """h = silu(a) * b with [a | b] = y the fused W1|W3 output; backward emits dy = [da | db]."""

    @staticmethod
    def forward(ctx, y):
        ctx.save_for_backward(y)
        return _hip().swiglu_fused_fwd(y)

    @staticmethod
    def backward(ctx, dh):
        (y,) = ctx.saved_tensors
        return _hip().swiglu_fused_bwd(dh.contiguous(), y)
