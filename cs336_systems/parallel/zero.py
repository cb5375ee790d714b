"""ZeRO-2 data parallelism with a sharded fused AdamW (a "distributed optimizer").

Beyond the reference: its sharded optimizer (``ddp_bucketed_overlapped_sharded.py:322-362``, here
:class:`~cs336_systems.parallel.ShardedOptimizer`) shards only the AdamW state, still all-reduces
every gradient, and then broadcasts every parameter from its owner. :class:`ZeroDDP` splits the
all-reduce into its two halves and puts the optimizer in between:

* **backward**: gradients land in persistent flat fp32 buckets (``param.grad`` is a view; the
  projection GEMMs write dW straight into them, as in :class:`DDPBucketed`). When a bucket is
  complete its **reduce-scatter** (``ReduceOp.AVG``) is issued asynchronously, so each rank ends
  backward with the averaged gradient of its 1/W shard of every bucket, overlapped with the rest of
  backward.
* **step**: one fused HIP AdamW launch over the rank's shards only (fp32 master = the rank's slice
  of the bucket's flat parameter buffer, ``m``/``v`` sized 1/W): the 30 B/param optimizer pass
  (≈10 ms for GPT-2 XL on one MI355X) shrinks W-fold.
* **param all-gather**, overlapped with the NEXT forward: every bucket's updated shard is
  all-gathered into the flat parameter buffer (the model's parameters are views of it)
  asynchronously right after the step, in forward order; a forward pre-hook on each module waits
  for exactly the buckets its parameters live in (a stream dependency on RCCL, not a host wait),
  then refreshes that bucket's bf16 compute shadows with one cast.

Per step each rank moves (W-1)/W of the fp32 gradient bytes (reduce-scatter) plus (W-1)/W of the
*bf16* parameter bytes (all-gather of the compute shadows, ``gather_dtype="auto"`` with
``bf16_shadows``): 6 B/param instead of an all-reduce's 8, the optimizer pass is 1/W as long, and
the parameter half of the traffic runs under the forward instead of the backward, where the xGMI
links are otherwise idle.
Buckets are padded to a multiple of W elements (pad elements stay zero through AdamW).
"""

from __future__ import annotations

import torch
import torch.distributed as dist
import torch.nn as nn

from ..models.fused import _SHADOW, _attach_transposed, _transpose_weight, dw_stream_for, mark_shadow_synced, refresh_transposed, sync_dw_stream
from ..ops.adamw import FusedAdamW, multi_tensor_l2norm
from ..utils.profiling import annotate
from .comm import broadcast_module_, supports_avg
from .ddp import DEFAULT_BUCKET_MB, _unique_params, bucket_params


class _ZBucket:
    __slots__ = ("idx", "params", "pbuf", "gbuf", "sbuf", "shard", "gshard", "master", "staged", "pending",
                 "launched", "rs", "ag", "bf16", "wbuf", "wshard")

    def __init__(self, idx, params, pbuf, gbuf, sbuf, shard, gshard, master, staged, bf16=False):
        self.idx, self.params, self.pbuf, self.gbuf, self.sbuf = idx, params, pbuf, gbuf, sbuf
        self.bf16 = bf16  # the parameter all-gather moves the bf16 compute shadows, not fp32 masters
        self.shard, self.gshard, self.master = shard, gshard, master
        self.staged = staged  # gloo + GPU tensors: collectives go through host copies
        self.pending = len(params)
        self.launched = False
        self.rs = None  # reduce-scatter work
        self.ag = None  # param all-gather work (True: a completed host-staged gather)
        self.wbuf = self.wshard = None  # low-precision wire copies of gbuf / gshard (comm_dtype)


class _ZeroAdamW(FusedAdamW):
    """FusedAdamW over the rank's flat shards; ``step`` also launches the param all-gathers and
    ``zero_grad`` resets the model's bucket gradients (the shard gradients stay attached)."""

    sharded_state = True  # one state file per rank in checkpoints (cs336_systems/checkpoint.py)

    def __init__(self, zero: "ZeroDDP", masters, **kw):
        super().__init__(masters, bf16_shadows=False, **kw)
        self._zero = zero

    def zero_grad(self, set_to_none: bool = True) -> None:
        self._zero.zero_grad(set_to_none=set_to_none)

    @torch.no_grad()
    def step(self, closure=None):
        self._zero._wait_all_gathers()  # a previous step's gathers must land before the shards change
        loss = super().step(closure)
        self._zero._launch_all_gathers()
        return loss


class ZeroDDP(nn.Module):
    """Data parallelism with reduce-scattered gradients and a sharded fused AdamW (module docstring).

    ``zero = ZeroDDP(model, lr=..., weight_decay=...)``; ``opt = zero.optimizer``; each step:
    ``opt.zero_grad()``, forward/backward through ``zero``, ``zero.finish_gradient_synchronization()``,
    optionally ``zero.clip_grad_norm_(c)``, ``opt.step()``. Parameters must be fp32 (the masters);
    ``bf16_shadows`` keeps a bf16 copy of every bucket that the model's GEMMs read under autocast.
    """

    def __init__(
        self,
        module: nn.Module,
        bucket_size_mb: float | None = DEFAULT_BUCKET_MB,
        process_group=None,
        broadcast: bool = True,
        lr: float = 1e-3,
        betas: tuple[float, float] = (0.9, 0.999),
        eps: float = 1e-8,
        weight_decay: float = 0.01,
        bf16_shadows: bool = False,
        overlap_param_gather: bool = True,
        gather_dtype: str = "auto",
        comm_dtype: torch.dtype | None = None,
        _collectives_at_world1: bool = False,
    ):
        super().__init__()
        self.module = module
        self.process_group = process_group
        self.world_size = dist.get_world_size(process_group)
        # tests: run the reduce-scatter / in-place all-gather path on a one-rank RCCL group too
        self._solo = self.world_size == 1 and not _collectives_at_world1
        self.rank = dist.get_rank(process_group)
        self._avg = supports_avg(process_group)
        self._gloo = dist.get_backend(process_group) == "gloo"
        self.overlap_param_gather = overlap_param_gather
        if broadcast:
            broadcast_module_(module, src=0, group=process_group)
        cap = float("inf") if bucket_size_mb is None else bucket_size_mb * 1024 * 1024
        params = [p for p in _unique_params(module) if p.requires_grad]
        for p in params:
            if p.dtype != torch.float32:
                raise TypeError(f"ZeroDDP keeps fp32 master weights; got a {p.dtype} parameter")
        W, r = self.world_size, self.rank
        self.buckets: list[_ZBucket] = []
        self._param_bucket: dict[nn.Parameter, _ZBucket] = {}
        self._views: dict[nn.Parameter, torch.Tensor] = {}
        # bf16 parameter gather: the forward of the projection weights reads only their bf16 shadows,
        # so only those go over the links (2 B/param instead of 4). Parameters read in fp32 by the
        # forward (embedding, norm gains) get buckets of their own, gathered in fp32, placed LAST in
        # the index order (their gradients complete last, and collectives are issued in index order).
        # The other ranks' fp32 masters of a bf16 bucket go stale; wait_for_params()/state_dict()
        # gather them on demand (checkpoints).
        if gather_dtype not in ("auto", "bf16", "fp32"):
            raise ValueError(f"gather_dtype must be auto|bf16|fp32, got {gather_dtype!r}")
        self._bf16_gather = bf16_shadows and not self._solo and gather_dtype in ("auto", "bf16")
        if self._bf16_gather:
            from ..models.transformer import Linear as _Linear

            lin = {id(m.weight) for m in module.modules() if isinstance(m, _Linear)}
            a = [p for p in params if id(p) in lin and p.dim() == 2]
            rest = [p for p in params if not (id(p) in lin and p.dim() == 2)]
            groups = [(ps, True) for ps in bucket_params(a, cap)] + [(ps, False) for ps in bucket_params(rest, cap)]
        else:
            groups = [(ps, False) for ps in bucket_params(params, cap)]
        self._masters_stale = False
        with torch.no_grad():
            for i, (ps, b16) in enumerate(groups):
                n = sum(p.numel() for p in ps)
                shard = (n + W - 1) // W
                dev = ps[0].device
                pbuf = torch.zeros(shard * W, device=dev, dtype=torch.float32)
                gbuf = torch.zeros_like(pbuf)
                sbuf = torch.zeros(shard * W, device=dev, dtype=torch.bfloat16) if bf16_shadows else None
                off = 0
                for p in ps:
                    k = p.numel()
                    pbuf[off : off + k].copy_(p.data.reshape(-1))
                    # re-home the parameter into the flat buffer (grouped units stay row-adjacent)
                    p.data = pbuf[off : off + k].view_as(p)
                    self._views[p] = gbuf[off : off + k].view_as(p)
                    p._cs336_grad_out = self._views[p]
                    if sbuf is not None and p.dim() == 2:
                        setattr(p, _SHADOW, sbuf[off : off + k].view_as(p))
                    off += k
                if sbuf is not None and _transpose_weight():
                    # Wᵀ shadows (K-major operand of the input-gradient GEMM), re-written from the
                    # gathered bf16 shadows once per step (refresh_transposed: one launch per run)
                    _attach_transposed([p for p in ps if p.dim() == 2])
                master = nn.Parameter(pbuf[r * shard : (r + 1) * shard])
                # one rank: the "shard" is the whole bucket, no collective runs and the update
                # kernel writes the bf16 shadows itself (as FusedAdamW does without ZeRO)
                gshard = gbuf if self._solo else torch.zeros(shard, device=dev, dtype=torch.float32)
                master.grad = gshard
                if self._solo and sbuf is not None:
                    setattr(master, _SHADOW, sbuf)
                elif b16:  # the update kernel writes this rank's shadow slice; the gather ships it
                    setattr(master, _SHADOW, sbuf[r * shard : (r + 1) * shard])
                b = _ZBucket(i, ps, pbuf, gbuf, sbuf, shard, gshard, master, self._gloo and dev.type == "cuda", b16)
                if comm_dtype is not None and comm_dtype != torch.float32 and not self._solo:
                    # gradients reduce-scattered in comm_dtype (half the bytes for bf16), cast back
                    # into the fp32 shard the update reads at finish_gradient_synchronization
                    b.wbuf = torch.empty(shard * W, device=dev, dtype=comm_dtype)
                    b.wshard = torch.empty(shard, device=dev, dtype=comm_dtype)
                self.buckets.append(b)
                for p in ps:
                    self._param_bucket[p] = b
                if sbuf is not None:
                    self._refresh_shadows(b)
        self.optimizer = _ZeroAdamW(self, [b.master for b in self.buckets], lr=lr, betas=betas, eps=eps,
                                    weight_decay=weight_decay)
        self._hooks = [p.register_post_accumulate_grad_hook(self._on_grad_ready) for p in params]
        # forward pre-hooks: wait for the all-gathers of the buckets a module's parameters live in
        self._fwd_hooks = []
        self._module_buckets: dict[int, list[int]] = {}
        for m in module.modules():
            mine = {self._param_bucket[p].idx for p in m.parameters(recurse=m is not module) if p in self._param_bucket}
            if mine:
                ids = sorted(mine, reverse=True)
                self._module_buckets[id(m)] = ids
                self._fwd_hooks.append(m.register_forward_pre_hook(lambda _m, _a, ids=ids: self._wait_buckets(ids)))
        # parameters read without their module's forward (the fused add+RMSNorm path of
        # BasicsTransformerLM reads ln2 / the next ln1 / ln_final gains directly): the model calls
        # this right before such a read, so those buckets are waited for too
        if hasattr(module, "register_param_read_hook"):
            module.register_param_read_hook(lambda m: self._wait_buckets(self._module_buckets.get(id(m), ())))
        self._next = 0  # next bucket to reduce-scatter (strict index order on every rank)
        self._issued: list[int] = []
        self.zero_grad(set_to_none=False)

    def forward(self, *inputs, **kwargs):
        return self.module(*inputs, **kwargs)

    # ---- gradients --------------------------------------------------------------------------
    def zero_grad(self, set_to_none: bool = True) -> None:
        """``set_to_none``: unset the model's grads (the GEMMs then write dW straight into the
        buckets, every other gradient is copied into its view once); else zero the buckets."""
        for b in self.buckets:
            if not set_to_none:
                b.gbuf.zero_()
            for p in b.params:
                p.grad = None if set_to_none else self._views[p]

    def on_train_batch_start(self) -> None:
        self.zero_grad(set_to_none=False)

    def _adopt(self, p: nn.Parameter) -> None:
        v = self._views[p]
        g = p.grad
        if g is None:
            v.zero_()
        elif g.data_ptr() != v.data_ptr():
            v.copy_(g)
        p.grad = v

    def _on_grad_ready(self, p: nn.Parameter) -> None:
        b = self._param_bucket[p]
        self._adopt(p)
        b.pending -= 1
        # issue every leading complete bucket in index order: collectives pair by issue order, so
        # every rank must issue the same sequence (a bucket finishing early waits its turn)
        while self._next < len(self.buckets) and self.buckets[self._next].pending == 0:
            self._launch_rs(self.buckets[self._next])
            self._next += 1

    def _launch_rs(self, b: _ZBucket) -> None:
        b.launched = True
        if b.idx == 0:
            self._issued.clear()
        self._issued.append(b.idx)
        if self._solo:
            return
        op = dist.ReduceOp.AVG if self._avg else dist.ReduceOp.SUM
        with annotate(f"comm.rs{b.idx}"):
            if b.staged:  # gloo cannot reduce-scatter HIP tensors: stage on the host
                sync_dw_stream()
                wdt = b.wbuf.dtype if b.wbuf is not None else torch.float32
                out = torch.empty(b.shard, dtype=wdt)
                dist.reduce_scatter_tensor(out, b.gbuf.to(wdt).cpu(), op=op, group=self.process_group)
                b.gshard.copy_(out)
                return
            src, dst = (b.gbuf, b.gshard) if b.wbuf is None else (b.wbuf, b.wshard)
            side = dw_stream_for(b.gbuf)
            if side is None:
                if b.wbuf is not None:
                    b.wbuf.copy_(b.gbuf)
                b.rs = dist.reduce_scatter_tensor(dst, src, op=op, group=self.process_group, async_op=True)
                return
            # weight gradients may still be in flight on the dW side stream: issue from that stream
            # once it has caught up with the main stream (as DDPBucketed._all_reduce), so the main
            # stream keeps running backward instead of waiting for every dW GEMM issued so far
            side.wait_stream(torch.cuda.current_stream(b.gbuf.device))
            with torch.cuda.stream(side):
                if b.wbuf is not None:
                    b.wbuf.copy_(b.gbuf)
                b.rs = dist.reduce_scatter_tensor(dst, src, op=op, group=self.process_group, async_op=True)

    def launch_order(self) -> list[int]:
        """Bucket indices in the order their reduce-scatters were issued last step (tests)."""
        return list(self._issued)

    def remove_hooks(self) -> None:
        """Unregister the gradient and forward-pre hooks (see ``DDPBucketed.remove_hooks``)."""
        for h in list(self.__dict__.get("_hooks", ())) + list(self.__dict__.get("_fwd_hooks", ())):
            h.remove()
        self.__dict__["_hooks"], self.__dict__["_fwd_hooks"] = [], []

    def finish_gradient_synchronization(self) -> None:
        for b in self.buckets[self._next :]:  # buckets with unused parameters: continue the order
            for p in b.params:
                self._adopt(p)
            self._launch_rs(b)
        self._next = 0
        for b in self.buckets:
            if b.rs is not None:
                b.rs.wait()
                b.rs = None
                if b.wshard is not None:
                    b.gshard.copy_(b.wshard)
            if not self._avg and self.world_size > 1:
                b.gshard.div_(self.world_size)
            b.launched = False
            b.pending = len(b.params)

    @torch.no_grad()
    def clip_grad_norm_(self, max_norm: float) -> torch.Tensor:
        """Global L2 norm over the reduced gradient (sum of shard norms² across ranks), then scale
        the shards by ``min(1, max_norm / (norm + 1e-6))`` (reference ``nn_utils.py:20-30``)."""
        sq = multi_tensor_l2norm([b.gshard for b in self.buckets]).float() ** 2
        if self._gloo and sq.is_cuda:
            h = sq.cpu()
            dist.all_reduce(h, group=self.process_group)
            sq.copy_(h)
        else:
            dist.all_reduce(sq, group=self.process_group)
        norm = sq.sqrt()
        scale = torch.clamp(max_norm / (norm + 1e-6), max=1.0)
        for b in self.buckets:
            b.gshard.mul_(scale)
        return norm

    # ---- parameters -------------------------------------------------------------------------
    def _launch_all_gathers(self) -> None:
        if self._solo:  # the update wrote the parameters and their shadows in place
            for b in self.buckets:
                for p in b.params:
                    if b.sbuf is not None and p.dim() == 2:
                        mark_shadow_synced(p)
                if b.sbuf is not None:
                    refresh_transposed(b.params)
            return
        for b in reversed(self.buckets):  # forward order: the last buckets hold the first layers
            with annotate(f"comm.ag{b.idx}"):
                b.ag = self._gather(b.sbuf if b.bf16 else b.pbuf, b.shard, async_op=True)
        self._masters_stale = self._masters_stale or any(b.bf16 for b in self.buckets)
        if not self.overlap_param_gather:
            self._wait_all_gathers()

    def _gather(self, buf: torch.Tensor, shard: int, async_op: bool):
        """All-gather this rank's slice of ``buf`` into all of ``buf``: the work handle, or True for
        a completed host-staged gather (gloo cannot gather HIP tensors)."""
        own = buf[self.rank * shard : (self.rank + 1) * shard]
        if self._gloo and (buf.is_cuda or buf.dtype != torch.float32):
            # (bf16 travels as fp32 through gloo: exact both ways)
            full = torch.empty(buf.numel(), dtype=torch.float32)
            dist.all_gather_into_tensor(full, own.float().cpu(), group=self.process_group)
            buf.copy_(full)
            return True
        if self._gloo:  # CPU: gloo wants a separate input buffer
            w = dist.all_gather_into_tensor(buf, own.clone(), group=self.process_group, async_op=async_op)
        else:  # RCCL gathers in place: the input is this rank's slice of the output buffer
            w = dist.all_gather_into_tensor(buf, own, group=self.process_group, async_op=async_op)
        return w if async_op else True

    @torch.no_grad()
    def _gather_masters(self) -> None:
        """Bring the other ranks' fp32 masters of the bf16-gathered buckets up to date (blocking)."""
        if not self._masters_stale:
            return
        self._wait_all_gathers()
        for b in self.buckets:
            if b.bf16:
                w = self._gather(b.pbuf, b.shard, async_op=True)
                if w is not True:
                    w.wait()
        self._masters_stale = False

    def _wait_bucket(self, b: _ZBucket) -> None:
        if b.ag is None:
            return
        if b.ag is not True:
            b.ag.wait()
        b.ag = None
        if b.bf16:  # the gathered bytes ARE the shadows
            for p in b.params:
                mark_shadow_synced(p)
            refresh_transposed(b.params)
        elif b.sbuf is not None:
            self._refresh_shadows(b)

    def _wait_buckets(self, ids) -> None:
        for i in ids:
            self._wait_bucket(self.buckets[i])
        # a forward that reads the fp32 masters (no bf16 autocast: the shadows are not used) must
        # not see other ranks' stale masters after a bf16-only gather
        if self._masters_stale and not (torch.is_autocast_enabled("cuda") or torch.is_autocast_enabled("cpu")):
            self._gather_masters()

    def _wait_all_gathers(self) -> None:
        for b in reversed(self.buckets):
            self._wait_bucket(b)

    @torch.no_grad()
    def _refresh_shadows(self, b: _ZBucket) -> None:
        b.sbuf.copy_(b.pbuf)
        for p in b.params:
            if p.dim() == 2:
                mark_shadow_synced(p)
        refresh_transposed(b.params)

    def wait_for_params(self) -> None:
        """Make the current stream wait for every pending parameter all-gather and bring every fp32
        master up to date (before reading the full parameters outside a forward, e.g. for a
        checkpoint; with the bf16 gather this runs an fp32 all-gather of those buckets)."""
        self._wait_all_gathers()
        self._gather_masters()

    def state_dict(self, *args, **kwargs):
        self.wait_for_params()
        return self.module.state_dict(*args, **kwargs)

    def bucket_summary(self) -> list[dict]:
        return [dict(bucket=b.idx, n_params=len(b.params), mb=b.pbuf.numel() * 4 / 2**20, shard=b.shard,
                     gather="bf16" if b.bf16 else "fp32",
                     wire=str(b.wbuf.dtype if b.wbuf is not None else torch.float32).replace("torch.", ""),
                     wire_mb=b.pbuf.numel() * (b.wbuf.element_size() if b.wbuf is not None else 4) / 2**20)
                for b in self.buckets]
