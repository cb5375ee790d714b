"""Context (sequence) parallelism: ring attention over a process group.

The reference scales sequence length only through single-device FlashAttention-2 — whose backward
even materializes N x N ("no ring attention, context parallel or
Ulysses"). Here a sequence of N tokens is split over the W ranks of a group. Every token-local
part of the Transformer (embedding, RMSNorm, projections, SwiGLU, the loss) runs unchanged on the
rank's n = N/W tokens; only attention needs the other ranks' keys/values, and it gets them by
passing K/V chunks around a ring (P2P send/recv; RCCL over xGMI on MI355X, each hop one neighbour
link) while the rank's queries stay put:

* forward: at step s a rank attends its queries to the chunk that started s ranks upstream with
  the FA2 kernels (``fa_fwd``, which already returns the log-sum-exp) and merges the partial
  results in fp32 by their LSE, ``o = (o_a e^{l_a} + o_b e^{l_b}) / (e^{l_a} + e^{l_b})``; the next
  chunk's transfer is in flight during the current chunk's attention;
* backward: (K, V, dK, dV) travel the same ring. Each rank adds the gradient contribution of its
  queries to the visiting chunk's dK/dV — ``fa_bwd`` with the *final* O and LSE makes
  P = exp(S − LSE) exact for a partial key set — keeps dQ locally, and after W hops every chunk's
  dK/dV is back on its owner. Memory stays O(N/W) per rank; nothing N x N exists anywhere.

Causal work balance: with the ``"contiguous"`` layout (rank r holds tokens [r·n, (r+1)·n)) rank 0
attends one chunk and rank W−1 all W. The ``"zigzag"`` layout cuts the sequence into 2W
sub-chunks and gives rank r sub-chunks r and 2W−1−r, so every rank does the same causal work. A
(query sub-chunk i, key sub-chunk j) pair is full attention when j < i, causal when j == i and
skipped when j > i.

**Ulysses** (``layout="ulysses"``, DeepSpeed-Ulysses style) is the all-to-all alternative: tokens
are sharded contiguously, and around attention two all-to-alls switch the sharding from sequence to
heads and back — each rank attends H/W heads over the FULL sequence with one ordinary causal FA2
call (balanced by construction), so the communication is 2 x 3 (q, k, v) + 2 (o) all-to-alls of
n·H·D elements per layer, independent of W hops, at the price of H % W == 0. XL's 25 heads do not
divide by 2/4/8; the 2.7b model's 32 do.

Use: :func:`enable_context_parallel` on a :class:`~cs336_systems.models.BasicsTransformerLM`,
feed each rank ``shard_sequence(tokens, rank, world, layout)`` (RoPE positions default to the
tokens' global positions), and average gradients over the group (any DP wrapper on the same group:
the per-rank mean losses average to the global mean because every rank holds the same number of
tokens). ``tests/test_context_parallel.py`` checks outputs and gradients against the
single-process model.
"""

from __future__ import annotations

import torch
import torch.distributed as dist
import torch.nn as nn

from ..ops._ext import use_hip
from ..ops.flash_attention import _tiled_backward, _tiled_forward, flash_attn_bwd, flash_attn_fwd

LAYOUTS = ("contiguous", "zigzag", "ulysses")


def _world_rank(group) -> tuple[int, int]:
    if not (dist.is_available() and dist.is_initialized()):
        return 1, 0
    return dist.get_world_size(group), dist.get_rank(group)


def _sub_ids(rank: int, world: int, layout: str) -> list[int]:
    """Global sub-chunk indices held by ``rank`` (in local order)."""
    if layout in ("contiguous", "ulysses"):
        return [rank]
    if layout == "zigzag":
        return [rank, 2 * world - 1 - rank]
    raise ValueError(f"unknown context-parallel layout {layout!r} (expected one of {LAYOUTS})")


def _n_sub(layout: str) -> int:
    return 2 if layout == "zigzag" else 1


def shard_sequence(x: torch.Tensor, rank: int, world: int, layout: str = "zigzag", dim: int = 1) -> torch.Tensor:
    """The part of ``x`` (sequence along ``dim``) that ``rank`` holds."""
    n = x.shape[dim]
    nsub = world * _n_sub(layout)
    if n % nsub:
        raise ValueError(f"sequence length {n} must be divisible by {nsub} for {layout} context parallelism over {world} ranks")
    c = n // nsub
    parts = [x.narrow(dim, i * c, c) for i in _sub_ids(rank, world, layout)]
    return torch.cat(parts, dim) if len(parts) > 1 else parts[0].contiguous()


def unshard_sequence(chunks: list[torch.Tensor], layout: str = "zigzag", dim: int = 1) -> torch.Tensor:
    """Inverse of :func:`shard_sequence`: ``chunks[r]`` is rank r's part."""
    world, S = len(chunks), _n_sub(layout)
    c = chunks[0].shape[dim] // S
    pieces: list[torch.Tensor | None] = [None] * (world * S)
    for r, t in enumerate(chunks):
        for j, gid in enumerate(_sub_ids(r, world, layout)):
            pieces[gid] = t.narrow(dim, j * c, c)
    return torch.cat(pieces, dim)


def sequence_positions(seq_len: int, rank: int, world: int, layout: str = "zigzag", device=None) -> torch.Tensor:
    """Global token positions of ``rank``'s part of a ``seq_len`` sequence (for RoPE)."""
    return shard_sequence(torch.arange(seq_len, device=device), rank, world, layout, dim=0)


# ------------------------------------------------------------------------------------------
# partial attention on (B, H, n, D) views: HIP FA2 kernels on GPU, tiled PyTorch on CPU
# ------------------------------------------------------------------------------------------
def _attn_fwd(q, k, v, causal: bool, scale: float):
    if use_hip(q):
        o, lse = flash_attn_fwd(q, k, v, causal, scale)
        return o, lse
    B, H, n, D = q.shape
    o, lse = _tiled_forward(q.reshape(B * H, n, D), k.reshape(B * H, -1, D), v.reshape(B * H, -1, D), causal, scale)
    return o.view(B, H, n, D), lse.view(B, H, n)


def _attn_bwd(do, q, k, v, o, lse, causal: bool, scale: float):
    if use_hip(q):
        return flash_attn_bwd(do, q, k, v, o, lse, causal, scale)
    B, H, n, D = q.shape
    m = k.shape[2]
    dq, dk, dv = _tiled_backward(
        q.reshape(B * H, n, D), k.reshape(B * H, m, D), v.reshape(B * H, m, D), o.reshape(B * H, n, D),
        lse.reshape(B * H, n), do.reshape(B * H, n, D), causal, scale,
    )
    return dq.view(B, H, n, D), dk.view(B, H, m, D), dv.view(B, H, m, D)


def _merge(acc_o: list, acc_l: list, i: int, o: torch.Tensor, lse: torch.Tensor) -> None:
    """Fold a partial (o, lse) over a disjoint key set into accumulator ``i`` (fp32)."""
    o, lse = o.float(), lse.float()
    if acc_o[i] is None:
        acc_o[i], acc_l[i] = o, lse
        return
    m = torch.maximum(acc_l[i], lse)
    a, b = torch.exp(acc_l[i] - m), torch.exp(lse - m)
    s = a + b
    acc_o[i] = (acc_o[i] * (a / s)[..., None]) + (o * (b / s)[..., None])
    acc_l[i] = m + torch.log(s)


class _RingXfer:
    """Send ``tensors`` to the next rank and receive the previous rank's (P2P, in flight until
    :meth:`wait`, which returns the received tensors). With gloo and GPU tensors (the one-GPU
    multi-rank rehearsal) the transfer is staged through host memory explicitly, so it is ordered
    with the kernels that produce and consume the buffers."""

    def __init__(self, tensors: list[torch.Tensor], group):
        world, rank = _world_rank(group)
        nxt, prv = (rank + 1) % world, (rank - 1) % world
        if group is not None:
            nxt, prv = dist.get_global_rank(group, nxt), dist.get_global_rank(group, prv)
        self.device = tensors[0].device
        self.staged = tensors[0].is_cuda and dist.get_backend(group) == "gloo"
        send = [t.cpu() for t in tensors] if self.staged else tensors
        self.bufs = [torch.empty_like(t) for t in send]
        ops = [dist.P2POp(dist.isend, t, nxt, group) for t in send]
        ops += [dist.P2POp(dist.irecv, b, prv, group) for b in self.bufs]
        self.reqs = dist.batch_isend_irecv(ops)

    def wait(self) -> list[torch.Tensor]:
        for r in self.reqs:
            r.wait()
        return [b.to(self.device) for b in self.bufs] if self.staged else self.bufs


class RingAttention(torch.autograd.Function):
    """Attention of this rank's queries against the whole (distributed) sequence.

    ``q, k, v``: (B, H, n, D) local parts in the ``layout`` order (:func:`shard_sequence` along the
    sequence dim). Returns the local (B, H, n, D) output."""

    @staticmethod
    def forward(ctx, q, k, v, group=None, causal: bool = True, layout: str = "zigzag"):
        world, rank = _world_rank(group)
        S = _n_sub(layout)
        n = q.shape[2]
        if n % S or k.shape[2] != n:
            raise ValueError("ring attention needs equal local q/k lengths divisible by the layout's sub-chunks")
        c = n // S
        scale = q.shape[-1] ** -0.5
        mine = _sub_ids(rank, world, layout)
        k, v = k.contiguous(), v.contiguous()
        acc_o: list = [None] * S
        acc_l: list = [None] * S
        cur_k, cur_v = k, v
        for step in range(world):
            src = (rank - step) % world
            xfer = _RingXfer([cur_k, cur_v], group) if step + 1 < world else None
            theirs = _sub_ids(src, world, layout)
            for qi in range(S):
                for kj in range(S):
                    gq, gk = mine[qi], theirs[kj]
                    if causal and gk > gq:
                        continue
                    o, lse = _attn_fwd(
                        q[:, :, qi * c : (qi + 1) * c], cur_k[:, :, kj * c : (kj + 1) * c],
                        cur_v[:, :, kj * c : (kj + 1) * c], causal and gk == gq, scale,
                    )
                    _merge(acc_o, acc_l, qi, o, lse)
            if xfer is not None:
                cur_k, cur_v = xfer.wait()
        out = torch.cat([a.to(q.dtype) for a in acc_o], dim=2) if S > 1 else acc_o[0].to(q.dtype)
        ctx.save_for_backward(q, k, v, out, *[l.contiguous() for l in acc_l])
        ctx.group, ctx.causal, ctx.layout, ctx.scale = group, causal, layout, scale
        return out

    @staticmethod
    def backward(ctx, dout):
        q, k, v, out, *lses = ctx.saved_tensors
        group, causal, layout, scale = ctx.group, ctx.causal, ctx.layout, ctx.scale
        world, rank = _world_rank(group)
        S = _n_sub(layout)
        c = q.shape[2] // S
        mine = _sub_ids(rank, world, layout)
        if dout.stride(-1) != 1:
            dout = dout.contiguous()
        dq = torch.zeros(q.shape, dtype=torch.float32, device=q.device)
        cur_k, cur_v = k, v
        cur_dk = torch.zeros(k.shape, dtype=torch.float32, device=k.device)
        cur_dv = torch.zeros(v.shape, dtype=torch.float32, device=v.device)
        for step in range(world):
            src = (rank - step) % world
            kv_xfer = _RingXfer([cur_k, cur_v], group) if step + 1 < world else None
            theirs = _sub_ids(src, world, layout)
            for qi in range(S):
                qs = slice(qi * c, (qi + 1) * c)
                for kj in range(S):
                    gq, gk = mine[qi], theirs[kj]
                    if causal and gk > gq:
                        continue
                    ks = slice(kj * c, (kj + 1) * c)
                    dq_p, dk_p, dv_p = _attn_bwd(
                        dout[:, :, qs], q[:, :, qs], cur_k[:, :, ks], cur_v[:, :, ks], out[:, :, qs], lses[qi],
                        causal and gk == gq, scale,
                    )
                    dq[:, :, qs] += dq_p.float()
                    cur_dk[:, :, ks] += dk_p.float()
                    cur_dv[:, :, ks] += dv_p.float()
            if world > 1:  # the visiting chunk's gradients move on with it; the last hop returns them home
                cur_dk, cur_dv = _RingXfer([cur_dk, cur_dv], group).wait()
            if kv_xfer is not None:
                cur_k, cur_v = kv_xfer.wait()
        return dq.to(q.dtype), cur_dk.to(k.dtype), cur_dv.to(v.dtype), None, None, None


def ring_attention(q, k, v, group=None, causal: bool = True, layout: str = "zigzag") -> torch.Tensor:
    return RingAttention.apply(q, k, v, group, causal, layout)


# ------------------------------------------------------------------------------------------
# Ulysses: all-to-all between sequence sharding and head sharding
# ------------------------------------------------------------------------------------------
def _all_to_all(x: torch.Tensor, group) -> torch.Tensor:
    """``all_to_all_single`` over dim 0 (W equal blocks); host-staged for gloo + GPU tensors."""
    if x.is_cuda and dist.get_backend(group) == "gloo":
        h = x.cpu()
        out = torch.empty_like(h)
        dist.all_to_all_single(out, h, group=group)
        return out.to(x.device)
    out = torch.empty_like(x)
    dist.all_to_all_single(out, x, group=group)
    return out


def _seq_to_head(x: torch.Tensor, group) -> torch.Tensor:
    """(B, H, n, D) with this rank's tokens -> (B, H/W, W·n, D) with this rank's heads."""
    world, _ = _world_rank(group)
    B, H, n, D = x.shape
    send = x.reshape(B, world, H // world, n, D).permute(1, 0, 2, 3, 4).contiguous()  # block j -> rank j
    recv = _all_to_all(send, group)  # block i = rank i's tokens of my heads
    return recv.permute(1, 2, 0, 3, 4).reshape(B, H // world, world * n, D)


def _head_to_seq(y: torch.Tensor, group) -> torch.Tensor:
    """Inverse of :func:`_seq_to_head`."""
    world, _ = _world_rank(group)
    B, h, N, D = y.shape
    n = N // world
    send = y.reshape(B, h, world, n, D).permute(2, 0, 1, 3, 4).contiguous()  # block j = rank j's tokens
    recv = _all_to_all(send, group)  # block i = head group i of my tokens
    return recv.permute(1, 0, 2, 3, 4).reshape(B, world * h, n, D)


class _SeqToHead(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, group):
        ctx.group = group
        return _seq_to_head(x, group)

    @staticmethod
    def backward(ctx, g):
        return _head_to_seq(g.contiguous(), ctx.group), None


class _HeadToSeq(torch.autograd.Function):
    @staticmethod
    def forward(ctx, y, group):
        ctx.group = group
        return _head_to_seq(y, group)

    @staticmethod
    def backward(ctx, g):
        return _seq_to_head(g.contiguous(), ctx.group), None


def ulysses_attention(q, k, v, group=None, causal: bool = True) -> torch.Tensor:
    """Attention of this rank's contiguous token block (``q, k, v``: (B, H, n, D)) against the whole
    sequence: all-to-all to head sharding, one FA2 call over the full sequence, all-to-all back."""
    from ..ops.flash_attention import flash_attention

    world, _ = _world_rank(group)
    if q.shape[1] % world:
        raise ValueError(f"Ulysses needs the head count ({q.shape[1]}) divisible by the group size ({world})")
    qh, kh, vh = (_SeqToHead.apply(t, group) for t in (q, k, v))
    return _HeadToSeq.apply(flash_attention(qh, kh, vh, causal), group)


def enable_context_parallel(model: nn.Module, group=None, layout: str = "zigzag") -> nn.Module:
    """Switch every attention module of ``model`` to ring attention (or Ulysses all-to-all attention,
    ``layout="ulysses"``) over ``group``. The model then
    expects each rank's :func:`shard_sequence` part of the tokens; RoPE positions default to the
    global positions of those tokens."""
    if layout not in LAYOUTS:
        raise ValueError(layout)
    from ..models.transformer import CausalMultiHeadSelfAttention

    n = 0
    for m in model.modules():
        if isinstance(m, CausalMultiHeadSelfAttention):
            m.context_parallel = (group, layout)
            n += 1
    if n == 0:
        raise ValueError("model has no CausalMultiHeadSelfAttention modules")
    return model


def disable_context_parallel(model: nn.Module) -> nn.Module:
    from ..models.transformer import CausalMultiHeadSelfAttention

    for m in model.modules():
        if isinstance(m, CausalMultiHeadSelfAttention):
            m.context_parallel = None
    return model
