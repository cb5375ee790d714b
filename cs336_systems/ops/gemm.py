"""Projection GEMMs: hipBLASLt (``torch.mm``) or the hand-written MFMA kernel (``csrc/gemm/gemm.hip``).

``CS336_GEMM=hip`` routes every supported projection GEMM of :class:`FusedLinearFn` (forward
``X·Wᵀ``, input-grad ``dY·W``, weight-grad ``dYᵀ·X`` with fp32 output, optionally straight into a
DDP bucket) through the cs336 kernel; the default ``blas`` keeps hipBLASLt, which measured faster
on the XL shapes in round 1 (``profiles/r1_gemm_cs336_vs_hipblaslt.json``: the cs336 kernel reaches
60-100 % of hipBLASLt's TFLOPS; hipBLASLt picks stream-K 160×256 Tensile kernels for these shapes).
Unsupported shapes (tile divisibility, K % 64) always fall back to ``torch.mm``.

``CS336_GEMM=lt`` routes the same GEMMs through ``cs336::lt_gemm`` (``csrc/blas/lt_gemm.cpp``):
hipBLASLt with per-problem autotuning over the heuristic's top candidates (``CS336_LT_CANDIDATES``,
default 48), fp32 output included, which TunableOp does not cover. On the XL shapes the tuned pick
is within noise of ``torch.mm``'s on most GEMMs and 1.1-1.5x faster on a few fp32-output weight
gradients (``profiles/r1_lt_gemm_sweep*.json``), so ``blas`` stays the default.

``CS336_GEMM=best`` takes the fastest per problem of hipBLASLt's default pick (``torch.mm``), the
autotuned ``lt_gemm`` and the cs336 MFMA GEMM (where its tiling takes the shape): the first time a
(kind, shapes, strides, output) problem is seen outside graph capture, each applicable candidate is
timed on it (HIP events on the current stream) and the winner is cached for the process
(``gemm_choices`` / ``gemm_timings``). The round-1 sweeps show why no single one is right: ``lt`` wins
1.2x on the QKV GEMMs and the lm_head weight gradient but loses 1.2x on the W1|W3 weight gradient from
``Xᵀ``; the cs336 GEMM wins the o-projection forward (967 vs 886 TFLOP/s).

``concurrent_safe=True`` (weight-gradient GEMMs issued on the dW side stream, i.e. possibly beside
another GEMM) runs the cs336 MFMA GEMM: every workgroup owns whole output tiles and never waits for
another workgroup. hipBLASLt cannot be used there: on gfx950 2198 of the 2199 solutions of this
problem type are stream-K kernels (``scripts/lt_dp_probe.py``), which keep at most one workgroup per
CU and spin on flags set by later-dispatched workgroups of the same grid, so two of them sharing the
chip can deadlock (``csrc/blas/lt_gemm.cpp``, ``profiles/r2_streamk_hang.md``).
:func:`dw_concurrent_ok` says whether a weight gradient can go to the side stream at all.
"""

from __future__ import annotations

import os

import torch

from ._ext import ext_available, ops


def hip_gemm_enabled() -> bool:
    return _mode() == "hip"


def lt_gemm_enabled() -> bool:
    """``lt`` or ``best`` (the autotuned hipBLASLt op may be used)."""
    return _mode() in ("lt", "best")


def _mode(dw: bool = False) -> str:
    """GEMM implementation mode; ``dw``: for the weight-gradient GEMMs, where ``CS336_GEMM_DW``
    (if set) overrides ``CS336_GEMM`` — their fp32-output, long-K, small-output problems are the
    ones hipBLASLt's default pick serves worst."""
    m = os.environ.get("CS336_GEMM", "blas").lower()
    if dw:
        m = os.environ.get("CS336_GEMM_DW", m).lower()
    return m if m in ("lt", "best", "hip") and ext_available() else "blas"


_BEST: dict = {}
_TABLE: dict | None = None
TABLE_FILE = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tuning", "gemm_table_mi355x.json")


def selection_table() -> dict:
    """Committed per-problem picks (``cs336_systems/tuning/gemm_table_mi355x.json``, produced on
    MI355X by ``scripts/gemm_table.py`` from a ``CS336_GEMM_REPORT``): problem key -> implementation.
    Every rank and every box loads the same file, so ``best`` mode picks the same kernels everywhere
    and times nothing for the shapes it covers. ``CS336_GEMM_TABLE=0`` ignores it, ``=path`` loads
    another file."""
    global _TABLE
    if _TABLE is None:
        path = os.environ.get("CS336_GEMM_TABLE", TABLE_FILE)
        _TABLE = {}
        pins: list = []
        if path != "0" and os.path.exists(path):
            import json

            with open(path) as f:
                doc = json.load(f)
            _TABLE = dict(doc.get("entries", {}))
            pins = list(doc.get("lt_pins", []))
        if ext_available():
            # the autotuned hipBLASLt op takes the committed candidate (no per-process timing), and in a
            # multi-rank job an unpinned problem takes the heuristic's first choice instead of timing
            for pin in pins:
                m, n, k, at, bt, oc, idx, name = pin.split(",", 7)
                ops().lt_gemm_pin(int(m), int(n), int(k), at == "1", bt == "1", int(oc), int(idx), name)
            ops().lt_gemm_set_no_timing(_multi_rank())
    return _TABLE


def _multi_rank() -> bool:
    import torch.distributed as dist

    return dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1


def _time_ms(fn, reps: int = 5) -> float:
    fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    e1.synchronize()
    return e0.elapsed_time(e1) / reps


def _pick(kind: str, a: torch.Tensor, b: torch.Tensor, out: torch.Tensor | None, cands: dict) -> str:
    """``best`` mode: the committed table's pick for this problem (:func:`selection_table`); for a
    problem the table does not cover, the fastest of ``cands`` (name -> zero-arg launcher), timed
    once with HIP events on the current stream and cached ("blas" on near-ties, within 3 %). Never
    timed while a HIP graph is being captured, nor in a multi-rank job: per-process timing races
    could give ranks different kernels, and a timing run inside a DDP backward would sit beside
    in-flight all-reduces -- unseen problems run hipBLASLt's default there."""
    key = (kind, tuple(a.shape), a.stride(), tuple(b.shape), b.stride(),
           None if out is None else (out.dtype, out.stride()))
    hit = _BEST.get(key)
    if hit is None:
        t = selection_table().get(str(key))
        if t is None:
            # the same problem with other leading dimensions (ZeRO flat buffers put a group's Wᵀ in a
            # wider run: (2560, 20480) with ld 665360 on the 2.7b): the table's dense-layout pick
            t = selection_table().get(str(_dense_key(key)))
        if t is not None and t in cands:
            t = _multi_rank_safe(t, cands)
            _BEST[key] = t
            _BEST_TIMES[key] = {"table": t}
            return t
        if torch.cuda.is_current_stream_capturing():
            return "blas"
        if _multi_rank():
            t = _multi_rank_safe("blas", cands)
            _BEST[key] = t
            _BEST_TIMES[key] = {"untimed_multi_rank": t}
            return t
        # the partials of a split-K candidate are extra memory at the selection step (first step,
        # inside backward): time one only with room to spare; free memory is queried
        # here, on a cache miss, not on every call
        if any(hasattr(fn, "partial_bytes") for fn in cands.values()):
            free = torch.cuda.mem_get_info()[0]
            # only the split-K candidates are filtered: "blas" (and any candidate without partials)
            # always stays, so the comparison below never runs on an empty or blas-less set
            cands = {n: fn for n, fn in cands.items()
                     if not hasattr(fn, "partial_bytes") or fn.partial_bytes + (4 << 30) <= free}
        times = {name: _time_ms(fn) for name, fn in cands.items()}
        best = min(times, key=times.get)
        hit = _BEST[key] = best if times[best] < 0.97 * times["blas"] else "blas"
        _BEST_TIMES[key] = times
    return hit


_BEST_TIMES: dict = {}


def _multi_rank_safe(pick: str, cands: dict) -> str:
    """In a multi-rank job a hipBLASLt pick ("lt" / "blas") is replaced by a cs336 kernel where one
    applies (gemm8, else the older cs336 GEMM): hipBLASLt's picks for these shapes are stream-K
    kernels whose workgroups wait on later workgroups of their grid, the hazard beside RCCL
    collectives that ``cs336_systems/rccl_env.py`` describes, while every cs336 workgroup owns whole
    tiles and never waits for another. It costs the 2.7b table's four hipBLASLt picks 1-10 % each
    (``profiles/r5_gemm_2p7b.md``) and only in multi-rank runs; single-GPU runs keep the fastest."""
    if pick in ("lt", "blas") and _multi_rank():
        for alt in ("g8", "cs336"):
            if alt in cands:
                return alt
    return pick


def _dense_key(key: tuple) -> tuple:
    """``key`` with every operand's row stride set to its row length (unit column stride kept)."""
    kind, ash, ast, bsh, bst, out = key

    def dense(shape, stride):
        return (shape[1], 1) if len(shape) == 2 and stride[-1] == 1 else stride

    return (kind, ash, dense(ash, ast), bsh, dense(bsh, bst), out)


def gemm_choices() -> dict:
    """``best`` mode decisions so far: problem key -> winning implementation ("blas", "lt" or
    "cs336") and the measured ms of every candidate (``gemm_timings``)."""
    return dict(_BEST)


def gemm_timings() -> dict:
    return dict(_BEST_TIMES)


def _lt_ok(*ts) -> bool:
    return all(t.is_cuda and t.dim() == 2 and t.stride(1) == 1 for t in ts) and ts[0].dtype == torch.bfloat16 and ts[1].dtype == torch.bfloat16


def _ok(a, b, ta, tb) -> bool:
    return a.is_cuda and a.dtype == torch.bfloat16 and b.dtype == torch.bfloat16 and ops().gemm_ok(a, b, ta, tb)


def _select(kind, a, b, out, blas, lt, cs336, dw: bool = False, extra: dict | None = None) -> str:
    """Implementation for this call: ``lt``/``hip`` modes force theirs where it applies, ``best``
    times the applicable ones (``None`` = not applicable) plus ``extra`` (name -> launcher, best
    mode only), ``blas`` is hipBLASLt's default."""
    mode = _mode(dw)
    if mode in ("lt", "best"):
        selection_table()  # loads the committed picks / lt pins once
    if mode == "lt" and lt is not None:
        return "lt"
    if mode == "hip" and cs336 is not None:
        return "cs336"
    if mode == "best":
        cands = {"blas": blas}
        if lt is not None:
            cands["lt"] = lt
        if cs336 is not None:
            cands["cs336"] = cs336
        cands.update(extra or {})
        return _pick(kind, a, b, out, cands) if len(cands) > 1 else "blas"
    return "blas"


def _aligned_rows(t: torch.Tensor) -> bool:
    return t.dim() == 2 and t.stride(1) == 1 and t.stride(0) % 8 == 0 and t.data_ptr() % 16 == 0


DMA_LIMIT = (1 << 31) - (1 << 20)  # gemm8 / gemm8w: one buffer descriptor per operand, 32-bit offsets


def gemm8_extents_ok(x: torch.Tensor, w: torch.Tensor) -> bool:
    """Both operand extents the gemm8 kernel addresses (256 rows of ``x``, all rows of ``w``) fit
    its 2 GiB DMA range (mirrors ``gemm8_extents_ok`` in csrc/bindings.cpp)."""
    k = x.shape[1]
    return (255 * x.stride(0) + k) * 2 < DMA_LIMIT and ((w.shape[0] - 1) * w.stride(0) + k) * 2 < DMA_LIMIT


def gemm8_ok(x: torch.Tensor, w: torch.Tensor, epi: int = 0, half: int = 0) -> bool:
    """Whether the gemm8 NT kernel (``csrc/gemm/gemm8.hip``) takes ``x @ w.T``: bf16, row-major with
    16-B aligned rows, M % 256; epi 0: N and K multiples of 8 (partial last tiles masked); epi 1-3:
    K % 64, N a multiple of 320 or 256 (epi 1: half of 160 or 128); operand extents < 2 GiB."""
    return (
        x.is_cuda
        and x.dtype == torch.bfloat16
        and w.dtype == torch.bfloat16
        and _aligned_rows(x)
        and _aligned_rows(w)
        and x.shape[1] == w.shape[1]
        and ext_available()
        and ops().gemm8_ok(x.shape[0], w.shape[0], x.shape[1], epi, half)
        and gemm8_extents_ok(x, w)
    )


def gemm8(x: torch.Tensor, w: torch.Tensor) -> torch.Tensor:
    out = torch.empty(x.shape[0], w.shape[0], device=x.device, dtype=torch.bfloat16)
    ops().gemm8(x, w, out, 0, 0, None, None, 0)
    return out


def gemm8_swiglu_fwd(x: torch.Tensor, w13: torch.Tensor) -> tuple[torch.Tensor, torch.Tensor]:
    """``y = x @ [w1; w3].T`` and ``h = silu(y_a) * y_b`` from one kernel (SwiGLU gate in the GEMM
    epilogue): returns (y, h)."""
    half = w13.shape[0] // 2
    y = torch.empty(x.shape[0], 2 * half, device=x.device, dtype=torch.bfloat16)
    h = torch.empty(x.shape[0], half, device=x.device, dtype=torch.bfloat16)
    ops().gemm8(x, w13, y, 1, 0, h, None, half)
    return y, h


def gemm8_swiglu_bwd(dy: torch.Tensor, w2t: torch.Tensor, y: torch.Tensor) -> torch.Tensor:
    """``[da | db]`` from ``dh = dy @ w2t.T`` (never stored) and the saved ``y = [a | b]``: the W2
    input gradient with the SwiGLU backward in its epilogue."""
    half = w2t.shape[0]
    out = torch.empty(dy.shape[0], 2 * half, device=dy.device, dtype=torch.bfloat16)
    ops().gemm8(dy, w2t, out, 2, 0, None, y, half)
    return out


def qkv_rope_enabled() -> bool:
    """Whether the fused QKV forward applies RoPE in the GEMM's store (gemm8 epi 3): the cs336 GEMMs
    are in use (``best`` / ``hip`` modes) and ``CS336_QKV_ROPE`` is not ``0``."""
    return os.environ.get("CS336_QKV_ROPE", "1") != "0" and _mode() in ("best", "hip")


def gemm8_rope(x: torch.Tensor, w: torch.Tensor, cos: torch.Tensor, sin: torch.Tensor, pos: torch.Tensor | None,
               seq: int, rope_cols: int, dhead: int) -> torch.Tensor:
    """``x @ w.T`` with the columns below ``rope_cols`` (the q|k heads of a fused QKV projection)
    rotated by RoPE in the GEMM's store; ``pos``: int64 position per row, or None (row % seq)."""
    out = torch.empty(x.shape[0], w.shape[0], device=x.device, dtype=torch.bfloat16)
    ops().gemm8_rope(x, w, out, cos, sin, pos, seq, rope_cols, dhead)
    return out


def mm_nt(x: torch.Tensor, w: torch.Tensor) -> torch.Tensor:
    """``x @ w.T`` (forward of a linear layer; the input gradient through a Wᵀ shadow)."""
    mode = _mode()
    if mode == "blas":
        return torch.mm(x, w.t())
    blas = lambda: torch.mm(x, w.t())  # noqa: E731
    lt = (lambda: ops().lt_gemm(x, w, False, True, torch.bfloat16)) if _lt_ok(x, w) else None
    g8 = (lambda: gemm8(x, w)) if gemm8_ok(x, w) else None
    if mode == "hip":  # the hand-written kernels: gemm8 where it applies, else the older cs336 GEMM
        cs = g8 if g8 is not None else ((lambda: ops().gemm(x, w, False, True, torch.bfloat16, 0, 0, 0))
                                        if _ok(x, w, False, True) else None)
        return (cs or blas)()
    cs = (lambda: ops().gemm(x, w, False, True, torch.bfloat16, 0, 0, 0)) if _ok(x, w, False, True) else None
    extra = {"g8": g8} if g8 is not None else {}
    impls = {"blas": blas, "lt": lt, "cs336": cs, **extra}
    return impls[_select("nt", x, w, None, blas, lt, cs, extra=extra)]()


def mm_nn(dy: torch.Tensor, w: torch.Tensor) -> torch.Tensor:
    """``dy @ w`` (input gradient)."""
    if _mode() == "blas":
        return torch.mm(dy, w)
    blas = lambda: torch.mm(dy, w)  # noqa: E731
    lt = (lambda: ops().lt_gemm(dy, w, False, False, torch.bfloat16)) if _lt_ok(dy, w) else None
    cs = (lambda: ops().gemm(dy, w, False, False, torch.bfloat16, 0, 0, 0)) if _ok(dy, w, False, False) else None
    return {"blas": blas, "lt": lt, "cs336": cs}[_select("nn", dy, w, None, blas, lt, cs)]()


NO_STREAM_K = 1  # lt_gemm flag: data-parallel hipBLASLt solutions only (none exist on gfx950 today)


def dw_concurrent_ok(dy: torch.Tensor, x: torch.Tensor, xt_layout: bool) -> bool:
    """Whether ``dW = dyᵀ·x`` can run beside another GEMM: the cs336 GEMM (no inter-workgroup
    waits) must take the problem; the Xᵀ layout (K-major B) is not one of its orientations."""
    return not xt_layout and ext_available() and _ok(dy, x, True, False)


def _dw_concurrent(dy, x, out):
    """Weight gradient with the cs336 MFMA GEMM (data-parallel tiles, safe beside other GEMMs)."""
    if not _ok(dy, x, True, False):
        raise RuntimeError(f"cs336 GEMM does not take the weight gradient {tuple(dy.shape)}ᵀ·{tuple(x.shape)}")
    if out is None:
        return ops().gemm(dy, x, True, False, torch.float32, 0, 0, 0)
    ops().gemm_out(dy, x, True, False, out, False, 0, 0, 0)
    return out


def mm_tn_fp32_xt(dy: torch.Tensor, xt: torch.Tensor, out: torch.Tensor | None = None,
                  concurrent_safe: bool = False) -> torch.Tensor:
    """``dy.T @ xt.T`` with an fp32 result: the weight gradient from a token-contiguous ``Xᵀ``
    (K_in, tokens). hipBLASLt only (default or autotuned): its NT kernels are the fast ones for
    this layout and the cs336 GEMM has no (MN, K) orientation."""
    if concurrent_safe:
        raise RuntimeError("no concurrency-safe GEMM for the Xᵀ weight-gradient layout (dw_concurrent_ok)")
    if out is None:
        blas = lambda: torch.mm(dy.t(), xt.t(), out_dtype=torch.float32)  # noqa: E731
        lt = lambda: ops().lt_gemm(dy, xt, True, True, torch.float32)  # noqa: E731
    else:
        blas = lambda: torch.mm(dy.t(), xt.t(), out_dtype=torch.float32, out=out)  # noqa: E731
        lt = lambda: ops().lt_gemm_out(dy, xt, True, True, out)  # noqa: E731
    use_lt = _mode(True) in ("lt", "best") and _lt_ok(dy, xt) and (out is None or out.stride(1) == 1)
    if not use_lt:
        r = blas()
        return out if out is not None else r
    extra = {}
    if _mode(True) == "best" and dy.is_contiguous() and xt.is_contiguous():
        k, m = dy.shape
        n = xt.shape[0]
        extra = _splitk_cands(lambda sk: dy.view(sk, k // sk, m).transpose(1, 2),
                              lambda sk: xt.view(n, sk, k // sk).permute(1, 2, 0), k, m, n, out)
    impls = {"blas": blas, "lt": lt, **extra}
    r = impls[_select("tt32", dy, xt, out, blas, lt, None, dw=True, extra=extra)]()
    return out if out is not None else r


SPLITK_MAX_OUT = 32 << 20  # output elements up to which split-K candidates are timed (best mode)
SPLITK_MAX_PARTIAL_BYTES = 512 << 20  # fp32 partials of one split-K candidate


def _splitk_cands(a3_of, b3_of, k: int, m: int, n: int, out: torch.Tensor | None) -> dict:
    """Split-K candidates for a long-K, small-output fp32 weight gradient: the token dimension cut
    into S slices computed as one strided batched GEMM (S x more output tiles to spread over the
    256 CUs) whose fp32 partials are summed into the result. The o-projection dW (1600 x 1600 out,
    24576 tokens) fills only ~40 macro-tiles of 256 x 256 without it. ``a3_of(S)`` / ``b3_of(S)``
    give the (S, m, k/S) and (S, k/S, n) views."""
    if m * n > int(os.environ.get("CS336_SPLITK_MAX_OUT", SPLITK_MAX_OUT)) or os.environ.get("CS336_SPLITK", "1") == "0":
        return {}
    res = {}
    for sk in (2, 4, 8):
        if k % sk or (k // sk) % 64 or sk * m * n * 4 > SPLITK_MAX_PARTIAL_BYTES:
            continue

        def run(sk=sk):
            part = torch.bmm(a3_of(sk), b3_of(sk), out_dtype=torch.float32)
            return torch.sum(part, dim=0, out=out) if out is not None else part.sum(0)

        run.partial_bytes = sk * m * n * 4  # checked against free memory before it is timed (_pick)
        res[f"splitk{sk}"] = run
    return res


def mm_dyt_fp32(dyt: torch.Tensor, x: torch.Tensor, x_is_t: bool, out: torch.Tensor | None = None) -> torch.Tensor:
    """Weight gradient ``dyt @ x`` (``x_is_t``: ``dyt @ x.T``, x holding Xᵀ) with an fp32 result,
    from a token-contiguous ``dYᵀ`` (N_out, tokens). hipBLASLt default pick; ``best`` mode also times
    the autotuned hipBLASLt and the cs336 GEMM (both layouts have a K-major A operand)."""
    b = x.t() if x_is_t else x
    if out is None:
        blas = lambda: torch.mm(dyt, b, out_dtype=torch.float32)  # noqa: E731
    else:
        blas = lambda: torch.mm(dyt, b, out_dtype=torch.float32, out=out)  # noqa: E731
    if _mode(True) == "blas" or not dyt.is_cuda:
        r = blas()
        return out if out is not None else r
    lt_ok = _lt_ok(dyt, x) and (out is None or out.stride(1) == 1)
    if out is None:
        lt = (lambda: ops().lt_gemm(dyt, x, False, x_is_t, torch.float32)) if lt_ok else None
        cs = (lambda: ops().gemm(dyt, x, False, x_is_t, torch.float32, 0, 0, 0)) if _ok(dyt, x, False, x_is_t) else None
    else:
        lt = (lambda: ops().lt_gemm_out(dyt, x, False, x_is_t, out)) if lt_ok else None
        cs = (lambda: ops().gemm_out(dyt, x, False, x_is_t, out, False, 0, 0, 0)) if _ok(dyt, x, False, x_is_t) else None
    m, k = dyt.shape
    n = b.shape[1]
    if x_is_t:  # x = Xᵀ (n, k): slice s is x[:, s*kc:(s+1)*kc]ᵀ
        b3_of = lambda sk: x.view(n, sk, k // sk).permute(1, 2, 0)  # noqa: E731
    else:  # x (k, n) token-major
        b3_of = lambda sk: x.view(sk, k // sk, n)  # noqa: E731
    a3_of = lambda sk: dyt.view(m, sk, k // sk).permute(1, 0, 2)  # noqa: E731
    extra = _splitk_cands(a3_of, b3_of, k, m, n, out) if _mode(True) == "best" and dyt.is_contiguous() and (x.is_contiguous()) else {}
    impls = {"blas": blas, "lt": lt, "cs336": cs, **extra}
    r = impls[_select("dyt32" + ("t" if x_is_t else "n"), dyt, x, out, blas, lt, cs, dw=True, extra=extra)]()
    return out if out is not None else r


def mm_tn_fp32(dy: torch.Tensor, x: torch.Tensor, out: torch.Tensor | None = None,
               concurrent_safe: bool = False) -> torch.Tensor:
    """``dy.T @ x`` with an fp32 result (weight gradient), written into ``out`` when given."""
    if concurrent_safe:
        return _dw_concurrent(dy, x, out)
    if out is None:
        def blas():
            try:
                return torch.mm(dy.t(), x, out_dtype=torch.float32)
            except (TypeError, RuntimeError):
                return torch.mm(dy.t(), x).float()
    else:
        blas = lambda: torch.mm(dy.t(), x, out_dtype=torch.float32, out=out)  # noqa: E731
    if _mode(True) == "blas" or not dy.is_cuda:
        r = blas()
        return out if out is not None else r
    lt_ok = _lt_ok(dy, x) and (out is None or out.stride(1) == 1)
    if out is None:
        lt = (lambda: ops().lt_gemm(dy, x, True, False, torch.float32)) if lt_ok else None
        cs = (lambda: ops().gemm(dy, x, True, False, torch.float32, 0, 0, 0)) if _ok(dy, x, True, False) else None
    else:
        lt = (lambda: ops().lt_gemm_out(dy, x, True, False, out)) if lt_ok else None
        cs = (lambda: ops().gemm_out(dy, x, True, False, out, False, 0, 0, 0)) if _ok(dy, x, True, False) else None
    k, m = dy.shape
    n = x.shape[1]
    extra = {}
    if _mode(True) == "best" and dy.is_contiguous() and x.is_contiguous():
        extra = _splitk_cands(lambda sk: dy.view(sk, k // sk, m).transpose(1, 2), lambda sk: x.view(sk, k // sk, n),
                              k, m, n, out)
    impls = {"blas": blas, "lt": lt, "cs336": cs, **extra}
    r = impls[_select("tn32", dy, x, out, blas, lt, cs, dw=True, extra=extra)]()
    return out if out is not None else r


# ------------------------------------------------------------------------------------------
# weight gradients straight from token-major operands (csrc/gemm/gemm8w.hip)
# ------------------------------------------------------------------------------------------
def dw_g8w_enabled() -> bool:
    """``CS336_DW=g8w`` (default): projection weight gradients dW = dYᵀ·X run the cs336 gemm8w kernel
    on the token-major dY and X -- no dYᵀ / Xᵀ transposes in forward or backward; ``CS336_DW=blas``
    restores the hipBLASLt paths (best-mode table, Xᵀ / dYᵀ layouts)."""
    return os.environ.get("CS336_DW", "g8w") == "g8w" and ext_available()


# measured picks (scripts/gemm8w_bench.py, profiles/r3_gemm8w_bench.json): (tokens, N_out, K_in) ->
# (transposed roles, split-K count)
DW_PLANS: dict = {
    # XL (d 1600, d_ff 6400) at 24576 tokens, profiles/r3_gemm8w_bench.json (ms, vs hipBLASLt):
    (24576, 12800, 1600): (False, 1),  # W1|W3: 0.835 (default 1.27, lt 1.23, Xᵀ-layout blas 0.88)
    (24576, 1600, 6400): (True, 2),  # W2: 0.442 (lt 0.60; from dYᵀ 0.43 + its transpose)
    (24576, 4800, 1600): (False, 5),  # QKV: 0.377 (default 0.386)
    (24576, 1600, 1600): (False, 7),  # O: 0.139 (lt 0.224; split-K torch 0.164 + dYᵀ transpose)
    (24576, 10000, 1600): (False, 5),  # vocabulary head
    # per-GPU batch 96 (49152 tokens), profiles/r3_gemm8w_bench_49152.json: the same plans win
    (49152, 12800, 1600): (False, 1),  # W1|W3: 1.574 (lt 2.587)
    (49152, 1600, 6400): (True, 2),  # W2: 0.821 (lt 1.295)
    (49152, 4800, 1600): (False, 5),  # QKV: 0.678 (lt 0.950)
    (49152, 1600, 1600): (False, 7),  # O: 0.254 (lt 0.419)
    (49152, 10000, 1600): (False, 5),  # vocabulary head: 1.386 (lt 2.147)
    # per-GPU batch 102 (52224 tokens, the bench default from round 5): the 49152-token plans
    (52224, 12800, 1600): (False, 1),
    (52224, 1600, 6400): (True, 2),
    (52224, 4800, 1600): (False, 5),
    (52224, 1600, 1600): (False, 7),
    (52224, 10000, 1600): (False, 5),
}


def _dw_plan(T: int, n_out: int, k_in: int) -> tuple[bool, int] | None:
    """(transposed roles, split count) for dW [n_out, k_in] over T tokens: the measured plan, else a
    cost model -- padded row tiles of 256, column tiles of 320/256, quantisation over the 256 CUs,
    split-K slab traffic."""
    hit = DW_PLANS.get((T, n_out, k_in))
    if hit is not None:
        return hit
    best, best_t = None, float("inf")
    for trans in (False, True):
        M, N = (k_in, n_out) if trans else (n_out, k_in)
        bn = 320 if N % 320 == 0 else (256 if N % 256 == 0 else 0)
        if not bn or M % 8:
            continue
        tiles = -(-M // 256) * (N // bn)
        for sk in (1, 2, 3, 4, 5, 6, 7, 8):
            if T % 64 or (T // 64) < 4 * sk:
                continue
            wgs = tiles * sk
            eff = wgs / (-(-wgs // 256) * 256)
            t = 2.0 * T * (-(-M // 256) * 256) * N / (eff * 1.35e15)
            if sk > 1:
                t += (sk + 2) * M * N * 4 / 5.0e12
            if t < best_t:
                best, best_t = (trans, sk), t
    return best


def g8w_split_fits(T: int, sk: int, dy: torch.Tensor, x: torch.Tensor) -> bool:
    """One gemm8w split's operand extent (its token rows x the wider row stride) fits the kernel's
    2 GiB DMA range (csrc/bindings.cpp ``gemm8w``); a single split is cut into token chunks there."""
    rows = -(-(T // 64) // sk) * 64
    return rows * max(dy.stride(0), x.stride(0)) * 2 + max(dy.shape[1], x.shape[1]) * 2 < DMA_LIMIT


def dw_launch_plan(dy: torch.Tensor, x: torch.Tensor) -> tuple[bool, int]:
    """(transposed roles, splits) that :func:`mm_dw` launches: the measured / modelled plan, except
    that a split past the 2 GiB DMA range becomes one split, which the binding cuts into token
    chunks accumulated in place (e.g. a 50304-vocabulary head at 49152 tokens: 4.9 GB of dY)."""
    T = dy.shape[0]
    trans, sk = _dw_plan(T, dy.shape[1], x.shape[1])
    if sk > 1 and not g8w_split_fits(T, sk, dy, x):
        sk = 1
    return trans, sk


def dw_g8w_ok(dy: torch.Tensor, x: torch.Tensor) -> bool:
    return (dy.is_cuda and dy.dtype == torch.bfloat16 and x.dtype == torch.bfloat16 and dy.dim() == 2 and x.dim() == 2
            and dy.shape[0] == x.shape[0] and _aligned_rows(dy) and _aligned_rows(x) and dy.shape[0] % 64 == 0
            and dy.shape[1] % 8 == 0 and x.shape[1] % 8 == 0 and _dw_plan(dy.shape[0], dy.shape[1], x.shape[1]) is not None)


def mm_dw(dy: torch.Tensor, x: torch.Tensor, out: torch.Tensor | None = None, accumulate: bool = False) -> torch.Tensor:
    """``dy.T @ x`` with an fp32 result from token-major ``dy`` (T, N_out) and ``x`` (T, K_in) --
    written into ``out`` (e.g. a DDP bucket view; ``accumulate``: added to it) when given."""
    T, n_out, k_in = dy.shape[0], dy.shape[1], x.shape[1]
    trans, sk = dw_launch_plan(dy, x)
    a, b = (x, dy) if trans else (dy, x)
    if out is None:
        out = torch.empty(n_out, k_in, device=dy.device, dtype=torch.float32)
        accumulate = False
    direct = out.stride(1) == 1 and out.stride(0) % 4 == 0 and out.data_ptr() % 16 == 0
    if sk == 1:
        if direct:
            ops().gemm8w(a, b, out, 1, trans, accumulate, 0)
            return out
        tmp = torch.empty(n_out, k_in, device=dy.device, dtype=torch.float32)
        ops().gemm8w(a, b, tmp, 1, trans, False, 0)
        return out.add_(tmp) if accumulate else out.copy_(tmp)
    slabs = torch.empty(sk, n_out, k_in, device=dy.device, dtype=torch.float32)
    ops().gemm8w(a, b, slabs, sk, trans, False, 0)
    if direct and k_in % 4 == 0:
        ops().splitk_sum(slabs, out, accumulate)  # one pass over the slabs (torch.sum's dim-0 reduce: ~2.5x slower)
    elif accumulate:
        out.add_(slabs.sum(0))
    else:
        torch.sum(slabs, dim=0, out=out)
    return out
