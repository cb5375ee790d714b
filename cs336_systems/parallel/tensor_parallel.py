"""Megatron-style tensor parallelism for :class:`~cs336_systems.models.BasicsTransformerLM`.

Beyond the reference ("analytical only"). Inside every block the two matmul pairs
are split over the W ranks of a group so that each pair needs ONE all-reduce per direction:

* attention: q/k/v projections are **column-parallel** by heads (rank r keeps heads
  [r·H/W, (r+1)·H/W) — RoPE and FA2 are per-head, so the attention core runs unchanged on H/W
  heads), the output projection is **row-parallel** (its input columns of those heads); the
  partial outputs are summed by an all-reduce;
* SwiGLU: w1/w3 column-parallel over d_ff, w2 row-parallel, one all-reduce.

Autograd: the block input enters each split module through an identity whose backward all-reduces
dX (every rank computed dX from its shard of the weights), and the module output leaves through an
all-reduce whose backward is the identity. Both are forward hooks on the existing ``attn``/``ffn``
modules, so parameter names stay the reference's (the tensors are shards; :func:`gather_tp_state_dict`
rebuilds the full state dict). Embedding, norms and ``lm_head`` stay replicated and receive identical
gradients on every rank. The fused QKV / W1|W3 layouts are re-established on the shards, so the GPU
path keeps its grouped GEMMs. On MI355X the natural group is the 8 xGMI-connected GPUs of a node:
per block and direction TP moves 2 all-reduces of B·N·d_model activations.
"""

from __future__ import annotations

import torch
import torch.distributed as dist
import torch.nn as nn

from .comm import broadcast_module_


def _world_rank(group) -> tuple[int, int]:
    return dist.get_world_size(group), dist.get_rank(group)


def _all_reduce(t: torch.Tensor, group) -> torch.Tensor:
    t = t.contiguous()
    if t.is_cuda and dist.get_backend(group) == "gloo":  # gloo + HIP tensors: through the host
        h = t.cpu()
        dist.all_reduce(h, group=group)
        return h.to(t.device)
    t = t.clone()
    dist.all_reduce(t, group=group)
    return t


class _CopyToTP(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, group):
        ctx.group = group
        return x.view_as(x)

    @staticmethod
    def backward(ctx, g):
        return _all_reduce(g, ctx.group), None


class _ReduceFromTP(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, group):
        return _all_reduce(x, group)

    @staticmethod
    def backward(ctx, g):
        return g, None


def _keep_rows(p: nn.Parameter, sl: slice) -> None:
    p.data = p.data[sl].clone()


def _keep_cols(p: nn.Parameter, sl: slice) -> None:
    p.data = p.data[:, sl].contiguous()


@torch.no_grad()
def tensor_parallel_(model: nn.Module, group=None, broadcast: bool = True) -> nn.Module:
    """Shard every block of ``model`` in place over ``group`` (module docstring). Build the
    optimizer afterwards (the parameters change shape). Requires heads % W == 0 and d_ff % W == 0."""
    world, rank = _world_rank(group)
    if broadcast:
        broadcast_module_(model, src=0, group=group)
    layers = getattr(model, "layers", None)
    if layers is None:
        raise ValueError("tensor_parallel_ expects a BasicsTransformerLM-like model with .layers")
    for block in layers:
        attn, ffn = block.attn, block.ffn
        H, dk = attn.num_heads, attn.d_k
        if H % world:
            raise ValueError(f"{H} heads do not split over {world} tensor-parallel ranks")
        F = ffn.w1.weight.shape[0]
        if F % world:
            raise ValueError(f"d_ff {F} does not split over {world} tensor-parallel ranks")
        h, f = H // world, F // world
        heads = slice(rank * h * dk, (rank + 1) * h * dk)
        for lin in (attn.q_proj, attn.k_proj, attn.v_proj):
            _keep_rows(lin.weight, heads)
        _keep_cols(attn.output_proj.weight, heads)
        attn.num_heads = h
        ff = slice(rank * f, (rank + 1) * f)
        _keep_rows(ffn.w1.weight, ff)
        _keep_rows(ffn.w3.weight, ff)
        _keep_cols(ffn.w2.weight, ff)
        for m in (attn, ffn):
            m.register_forward_pre_hook(lambda _m, args, g=group: (_CopyToTP.apply(args[0], g), *args[1:]))
            m.register_forward_hook(lambda _m, _args, out, g=group: _ReduceFromTP.apply(out, g))
    if getattr(model, "_fused_layout", False):
        model.regroup_()
    model.tensor_parallel = (group, world)
    return model


@torch.no_grad()
def tp_clip_grad_norm_(model: nn.Module, max_norm: float, group=None) -> torch.Tensor:
    """Global gradient L2 norm of a tensor-parallel model (sharded gradients summed over the group,
    replicated ones counted once), then scale every gradient by ``min(1, max_norm / (norm + 1e-6))``."""
    sq_shard, sq_rep = None, None
    for name, p in model.named_parameters():
        if p.grad is None:
            continue
        s = p.grad.float().pow(2).sum()
        if _tp_split(name) is None:
            sq_rep = s if sq_rep is None else sq_rep + s
        else:
            sq_shard = s if sq_shard is None else sq_shard + s
    dev = next(model.parameters()).device
    sq_shard = torch.zeros((), device=dev) if sq_shard is None else sq_shard
    sq_rep = torch.zeros((), device=dev) if sq_rep is None else sq_rep
    norm = (_all_reduce(sq_shard.reshape(1), group)[0] + sq_rep).sqrt()
    scale = torch.clamp(max_norm / (norm + 1e-6), max=1.0)
    for p in model.parameters():
        if p.grad is not None:
            p.grad.mul_(scale.to(p.grad.dtype))
    return norm


def _tp_split(name: str) -> int | None:
    """Dim along which parameter ``name`` is sharded (0 rows, 1 columns), None if replicated."""
    if name.endswith(("attn.q_proj.weight", "attn.k_proj.weight", "attn.v_proj.weight", "ffn.w1.weight", "ffn.w3.weight")):
        return 0
    if name.endswith(("attn.output_proj.weight", "ffn.w2.weight")):
        return 1
    return None


def gather_tp_state_dict(model: nn.Module, group=None) -> dict:
    """The full (unsharded) state dict of a tensor-parallel model, on every rank (a collective)."""
    world, _ = _world_rank(group)
    out = {}
    for name, t in model.state_dict().items():
        dim = _tp_split(name)
        if dim is None or world == 1:
            out[name] = t.detach().clone()
            continue
        src = t.detach().contiguous()
        staged = src.is_cuda and dist.get_backend(group) == "gloo"
        if staged:
            src = src.cpu()
        parts = [torch.empty_like(src) for _ in range(world)]
        dist.all_gather(parts, src, group=group)
        out[name] = torch.cat(parts, dim).to(t.device)
    return out
