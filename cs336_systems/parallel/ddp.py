"""Data-parallel gradient synchronization, four variants.

=====================  ==================================================  ==========================
class                  mechanism                                           reference
=====================  ==================================================  ==========================
``NaiveDDP``           blocking all-reduce per parameter after backward   ``naive_ddp.py:173-267``
``FlatDDP``            one blocking all-reduce of a persistent flat grad   ``naive_ddp.py:444-634``
                       buffer (grads are views into it, no flatten copy)
``DDPIndividual``      async all-reduce per parameter from its post-        ``ddp_bucketed_overlapped_
                       accumulate-grad hook, overlapped with backward       sharded.py:217-248``
``DDPBucketed``        async all-reduce per bucket, overlapped with         ``…:251-318``
                       backward; buckets are persistent flat buffers and
                       ``param.grad`` is a *view* into them (zero-copy)
=====================  ==================================================  ==========================

MI355X/RCCL design notes:

* RCCL collectives run on the process group's own HIP stream; ProcessGroupNCCL records an event on
  the current (compute) stream before each launch, so an all-reduce issued from a grad hook runs
  concurrently with the rest of backward and ``Work.wait()`` only inserts a stream dependency (the
  host never blocks).
* With the nccl(=RCCL) backend the mean is taken by ``ReduceOp.AVG`` inside the collective; Gloo
  (CPU tests) uses SUM followed by one in-place divide per flat bucket.
* Bucket cap (``DEFAULT_BUCKET_MB``) — derived, and checked by emulation on one GPU (below); not yet
  measured on a multi-GPU RCCL node. The
  handout's overhead model prices ``n_b`` buckets of a gradient of ``s`` bytes at
  ``n_b·o + s/(w·n_b)``: a fixed launch/synchronisation cost ``o`` per collective plus the exposed
  all-reduce of the last bucket at algorithm bandwidth ``w``. It is minimal at
  ``bucket* = sqrt(s·w·o)``. For GPT-2 XL (s = 8.0 GB of fp32 gradients), an 8-rank RCCL ring over
  xGMI (bus bandwidth ≈ 300 GB/s of the 7 × 153 GB/s links ⇒ w = busbw / (2·7/8) ≈ 170 GB/s) and
  o ≈ 15-30 µs: bucket* ≈ 140-200 MB. Why 128 MB anyway: (1) the model is flat near its optimum —
  at o = 20 µs the model prices 128 MB at 2.00 ms and the optimum (165 MB) at 1.94 ms, a 0.06 ms
  difference; (2) the indivisible fused units of one XL layer (W1|W3 82 MB, W2 41 MB, QKV 31 MB, O
  10 MB, fp32) total ≈ 123 MB, so a 128 MB cap cuts the buckets at layer boundaries (74 buckets of
  61-127 MB, ``profiles/r3_multirank_rehearsal.jsonl``) and the first all-reduce starts after the
  last layer's backward instead of one and a half layers in; (3) the exposed tail of the last bucket
  stays ≈ 0.75 ms. ``bench.py`` at N > 1 appends an fp32 all-reduce sweep (1/10/100/1024 MB: algbw,
  busbw) to its JSON, from which ``w`` and ``o`` of the real node refit ``bucket*``. Measured by
  emulation on one GPU (``scripts/comm_emulation.py``, ``profiles/r5_comm_emulation.md``):
  RCCL-shaped occupants (16 or 32 channel blocks) held for each bucket's W = 8 ring time beside the
  real XL backward hide all 48 ms/step of communication at 128 MB (598.8 / 599.2 ms/step against
  599.7 for world-1 DDP), 512 MB exposes the last bucket (+4-8 ms), 32 MB with 32 channels loses
  52 ms. Round 6 re-ran it at the bench's batch 102 with occupants that also MOVE the ring's per-rank
  HBM bytes (``profiles/r6_comm_emulation.md``): 10.7-20.7 ms/step over world 1 at 32-128 MB, 512 MB
  +47-78 ms, and the backward-overlapped optimizer update slower beside the collectives in five of six
  configurations (so ``bench.py`` leaves it off at N > 1).
* World size 1 issues no collective at all (``_all_reduce``): RCCL runs ``ReduceOp.AVG`` on one rank
  as a separate scaling pass over every bucket (11.7 ms/step at XL), which no W > 1 ring runs. With it
  gone the one-rank wrapper is within 1 ms of the plain step (``profiles/r6_ddp_world1.md``).
* Unlike the reference, buckets hold only ``requires_grad`` parameters (no empty bucket 0, frozen
  params never block a flush).
* Collective order is identical on every rank: buckets are issued strictly in index order (a
  bucket that completes early waits for its predecessors), and a bucket whose parameters received
  no gradient on this rank is issued at ``finish_gradient_synchronization`` (zeros) in that same
  order. RCCL pairs collectives by issue order, so an out-of-order launch on one rank (e.g. a
  parameter unused on that rank only) would otherwise pair different buckets and hang.
"""

from __future__ import annotations

import torch
import torch.distributed as dist
import torch.nn as nn

from ..models.fused import dw_stream_for, sync_dw_stream
from ..utils.profiling import annotate
from .comm import broadcast_module_, supports_avg

DEFAULT_BUCKET_MB = 128.0


def _unique_params(module: nn.Module) -> list[nn.Parameter]:
    return list(module.parameters())  # parameters() already de-duplicates tied weights


def bucket_params(params: list[nn.Parameter], cap_bytes: float) -> list[list[nn.Parameter]]:
    """Greedy buckets over ``reversed(params)`` (≈ backward order) of at most ``cap_bytes``, never
    mixing dtypes/devices. The parameters of one fused group (the QKV / W1|W3 layout of
    models/fused.py, tagged ``_cs336_group``) form an indivisible unit laid out in storage order, so
    the grouped dW GEMM can write all of them into one contiguous region of the bucket. Untagged
    parameters are their own unit, even if they share a storage (e.g. after ZeRO-1 re-homed the whole
    model into one flat buffer: a storage key would then make the model a single bucket)."""

    def unit_key(p):
        g = getattr(p, "_cs336_group", None)
        return ("g", g) if g is not None else ("p", id(p))

    by_storage: dict = {}
    for p in params:
        by_storage.setdefault(unit_key(p), []).append(p)
    units, seen = [], set()
    for p in reversed(params):
        key = unit_key(p)
        if key in seen:
            continue
        seen.add(key)
        units.append(sorted(by_storage[key], key=lambda t: t.storage_offset()))
    groups: list[list[nn.Parameter]] = []
    cur: list[nn.Parameter] = []
    cur_bytes = 0
    for unit in units:
        nbytes = sum(p.numel() * p.element_size() for p in unit)
        p = unit[0]
        if cur and (cur_bytes + nbytes > cap_bytes or p.dtype != cur[0].dtype or p.device != cur[0].device):
            groups.append(cur)
            cur, cur_bytes = [], 0
        cur.extend(unit)
        cur_bytes += nbytes
    if cur:
        groups.append(cur)
    return groups


class _Done:
    """The handle of a collective that had nothing to do (world size 1): already complete."""

    def wait(self, timeout=None) -> bool:
        return True

    def is_completed(self) -> bool:
        return True


_DONE = _Done()


class _DDPBase(nn.Module):
    def __init__(self, module: nn.Module, process_group=None, broadcast: bool = True):
        super().__init__()
        self.module = module
        self.process_group = process_group
        self.world_size = dist.get_world_size(process_group)
        self.rank = dist.get_rank(process_group)
        self._avg = supports_avg(process_group)
        if broadcast:
            broadcast_module_(module, src=0, group=process_group)

    def forward(self, *inputs, **kwargs):
        return self.module(*inputs, **kwargs)

    def _all_reduce(self, t: torch.Tensor, async_op: bool):
        if self.world_size == 1:
            # the mean over one rank is the tensor itself: issue nothing. (RCCL runs ReduceOp.AVG on a
            # single rank as a separate scaling pass over every bucket -- 11.7 ms/step of XL, a pass that
            # W > 1 never runs because there the pre-multiply is fused into the ring, so a world-1
            # measurement of DDP's own cost would be dominated by it: profiles/r5_ddp_sweep_xl_world1.md)
            return _DONE if async_op else None
        op = dist.ReduceOp.AVG if self._avg else dist.ReduceOp.SUM
        # Weight gradients may still be in flight on the dW side stream (models/fused.py). Issue
        # the collective from that stream after it has caught up with the main stream: the
        # communication stream then waits for both, and the main stream keeps running backward.
        side = dw_stream_for(t)
        if side is None or not async_op:
            sync_dw_stream()
            return dist.all_reduce(t, op=op, group=self.process_group, async_op=async_op)
        side.wait_stream(torch.cuda.current_stream(t.device))
        with torch.cuda.stream(side):
            return dist.all_reduce(t, op=op, group=self.process_group, async_op=True)

    def _finish_mean(self, t: torch.Tensor) -> None:
        if not self._avg and self.world_size > 1:
            t.div_(self.world_size)

    def finish_gradient_synchronization(self) -> None:  # pragma: no cover - abstract
        raise NotImplementedError

    def remove_hooks(self) -> None:
        """Unregister the gradient hooks from the wrapped parameters. The hooks live in the
        parameters and hold this wrapper (bound methods), which holds the module: a
        wrapper dropped without this keeps the whole model alive for as long as its parameters are
        referenced anywhere -- the bench sweep built nine XL models, and seven stayed allocated
        (``profiles/r5_ddp_sweep_xl_world1.md``)."""
        for h in self.__dict__.get("_hooks", ()):
            h.remove()
        self.__dict__["_hooks"] = []


class NaiveDDP(_DDPBase):
    """Synchronous per-parameter all-reduce after backward (the handout's naive baseline)."""

    def finish_gradient_synchronization(self) -> None:
        for p in _unique_params(self.module):
            if p.requires_grad and p.grad is not None:
                self._all_reduce(p.grad, async_op=False)
                self._finish_mean(p.grad)


class FlatDDP(_DDPBase):
    """One blocking all-reduce over a persistent flat gradient buffer.

    ``param.grad`` tensors are views into ``self.flat`` (re-attached after ``zero_grad(set_to_none=
    True)``), so there is no flatten/unflatten copy (reference ``naive_ddp.py:543-553`` copies twice).
    """

    def __init__(self, module: nn.Module, process_group=None, broadcast: bool = True):
        super().__init__(module, process_group, broadcast)
        self._params = [p for p in _unique_params(module) if p.requires_grad]
        self._groups: dict[tuple, tuple[torch.Tensor, list]] = {}
        by_key: dict[tuple, list] = {}
        for p in self._params:
            by_key.setdefault((p.device, p.dtype), []).append(p)
        self._views = {}
        for key, ps in by_key.items():
            flat = torch.zeros(sum(p.numel() for p in ps), device=key[0], dtype=key[1])
            off = 0
            for p in ps:
                self._views[p] = flat[off : off + p.numel()].view_as(p)
                p._cs336_grad_out = self._views[p]  # GEMMs may write dW here directly
                off += p.numel()
            self._groups[key] = (flat, ps)
        self.zero_grad()

    def zero_grad(self, set_to_none: bool = False) -> None:
        for flat, ps in self._groups.values():
            flat.zero_()
            for p in ps:
                p.grad = self._views[p]

    def finish_gradient_synchronization(self) -> None:
        for flat, ps in self._groups.values():
            for p in ps:
                v = self._views[p]
                if p.grad is None:
                    v.zero_()
                elif p.grad.data_ptr() != v.data_ptr():
                    v.copy_(p.grad)
                p.grad = v
            with annotate("flat_allreduce"):
                self._all_reduce(flat, async_op=False)
            self._finish_mean(flat)


class DDPIndividual(_DDPBase):
    """Overlapped per-parameter all-reduce issued from post-accumulate-grad hooks."""

    def __init__(self, module: nn.Module, process_group=None, broadcast: bool = True):
        super().__init__(module, process_group, broadcast)
        self._handles: list[tuple[object, torch.Tensor]] = []
        self._hooks = []
        for p in _unique_params(module):
            if p.requires_grad:
                self._hooks.append(p.register_post_accumulate_grad_hook(self._on_grad_ready))

    def _on_grad_ready(self, p: torch.Tensor) -> None:
        with annotate("comm.param"):
            self._handles.append((self._all_reduce(p.grad, async_op=True), p.grad))

    def finish_gradient_synchronization(self) -> None:
        for h, g in self._handles:
            h.wait()
            self._finish_mean(g)
        self._handles.clear()


class _Bucket:
    __slots__ = ("idx", "params", "flat", "cflat", "pending", "handle", "launched")

    def __init__(self, idx: int, params: list, flat: torch.Tensor, cflat: torch.Tensor | None = None):
        self.idx = idx
        self.params = params
        self.flat = flat
        self.cflat = cflat  # low-precision wire copy (comm_dtype), or None
        self.pending = len(params)
        self.handle = None
        self.launched = False


class DDPBucketed(_DDPBase):
    """Overlapped bucketed all-reduce with persistent, zero-copy bucket buffers.

    Buckets are filled greedily over ``reversed(module.parameters())`` (≈ the order in which
    backward produces gradients) up to ``bucket_size_mb`` (``None`` → one unbounded bucket);
    a bucket never mixes dtypes/devices. Each parameter's ``.grad`` is a view into its bucket's
    flat buffer, so autograd accumulates straight into the communication buffer. If a caller
    resets grads to ``None`` (``optimizer.zero_grad()``), the projection GEMMs of the model write
    their fp32 dW directly into the bucket (``p._cs336_grad_out``; no memset, no accumulate add,
    no copy) and any other fresh gradient is copied into its view once by the hook.

    ``comm_dtype`` (e.g. ``torch.bfloat16``) puts the gradients on the wire in that dtype: each
    bucket is cast into a persistent wire buffer when it is issued, reduced there (AVG on RCCL),
    and cast back into the fp32 bucket at ``finish_gradient_synchronization``. Half the bytes per
    xGMI link for bf16 (the all-reduce is link-bound: 8 GB of fp32 gradients per GPT-2-XL step),
    for two extra elementwise passes over the bucket and bf16 rounding of the sum (the gradients
    themselves are already products of bf16 GEMM operands under autocast). Not combinable with the
    optimizer's per-bucket overlap callbacks (the reduced values reach the fp32 bucket only at
    finish). Default ``None``: the bucket's own dtype, as in the reference.
    """

    def __init__(self, module: nn.Module, bucket_size_mb: float | None = DEFAULT_BUCKET_MB, process_group=None,
                 broadcast: bool = True, comm_dtype: torch.dtype | None = None):
        super().__init__(module, process_group, broadcast)
        self.bucket_size_mb = bucket_size_mb
        self.comm_dtype = comm_dtype
        cap = float("inf") if bucket_size_mb is None else bucket_size_mb * 1024 * 1024
        params = [p for p in _unique_params(module) if p.requires_grad]
        groups = bucket_params(params, cap)
        self.buckets: list[_Bucket] = []
        self._param_bucket: dict[nn.Parameter, _Bucket] = {}
        self._views: dict[nn.Parameter, torch.Tensor] = {}
        for i, ps in enumerate(groups):
            flat = torch.zeros(sum(p.numel() for p in ps), device=ps[0].device, dtype=ps[0].dtype)
            off = 0
            for p in ps:
                self._views[p] = flat[off : off + p.numel()].view_as(p)
                self._param_bucket[p] = None  # filled below
                off += p.numel()
            wire = None
            if comm_dtype is not None and comm_dtype != flat.dtype:
                wire = torch.empty(flat.numel(), device=flat.device, dtype=comm_dtype)
            b = _Bucket(i, ps, flat, wire)
            self.buckets.append(b)
            for p in ps:
                self._param_bucket[p] = b
                # GEMM-output target: FusedLinearFn writes dW straight into the bucket when the
                # grad is unset (models/fused.py), so _adopt finds it already in place
                p._cs336_grad_out = self._views[p]
        self._hooks = [p.register_post_accumulate_grad_hook(self._on_grad_ready) for p in params]
        self._bucket_callbacks = []
        self._next = 0  # index of the next bucket to issue
        self._issued: list[int] = []
        self.zero_grad()

    def add_bucket_callback(self, fn) -> None:
        """``fn(params, work)`` runs right after a bucket's all-reduce is issued (``work`` is its
        async handle; with AVG the reduced gradients are final once it completes). Used by
        :class:`~cs336_systems.ops.FusedAdamW` to update each bucket during backward."""
        if any(b.cflat is not None for b in self.buckets):
            raise RuntimeError("per-bucket callbacks need full-precision buckets (comm_dtype=None)")
        self._bucket_callbacks.append(fn)

    def supports_bucket_callbacks(self) -> bool:
        return self._avg and all(b.cflat is None for b in self.buckets)

    # ---- grad buffer management -------------------------------------------------------------
    def zero_grad(self, set_to_none: bool = False) -> None:
        """Zero every bucket (one memset per bucket) and point each ``.grad`` at its view."""
        for b in self.buckets:
            b.flat.zero_()
            for p in b.params:
                p.grad = self._views[p]

    def on_train_batch_start(self) -> None:
        self.zero_grad()

    def _adopt(self, p: nn.Parameter) -> None:
        v = self._views[p]
        g = p.grad
        if g is None:
            v.zero_()
        elif g.data_ptr() != v.data_ptr():
            v.copy_(g)
        p.grad = v

    # ---- hooks ------------------------------------------------------------------------------
    def _launch(self, b: _Bucket) -> None:
        if b.idx == 0:
            self._issued.clear()
        self._issued.append(b.idx)
        with annotate(f"comm.bucket{b.idx}"):
            if b.cflat is not None:
                self._cast_into(b.cflat, b.flat)
                b.handle = self._all_reduce(b.cflat, async_op=True)
            else:
                b.handle = self._all_reduce(b.flat, async_op=True)
        b.launched = True
        for fn in self._bucket_callbacks:
            fn(b.params, b.handle)

    def _on_grad_ready(self, p: nn.Parameter) -> None:
        b = self._param_bucket[p]
        self._adopt(p)
        b.pending -= 1
        # issue every leading complete bucket, strictly in index order (same order on every rank)
        while self._next < len(self.buckets) and self.buckets[self._next].pending == 0:
            self._launch(self.buckets[self._next])
            self._next += 1

    def finish_gradient_synchronization(self) -> None:
        # buckets with parameters that got no gradient on this rank are reduced now, continuing the
        # index order
        for b in self.buckets[self._next :]:
            for p in b.params:
                self._adopt(p)
            self._launch(b)
        self._next = 0
        for b in self.buckets:
            b.handle.wait()
            if b.cflat is not None:
                b.flat.copy_(b.cflat)
            self._finish_mean(b.flat)
            b.handle = None
            b.launched = False
            b.pending = len(b.params)

    @staticmethod
    def _cast_into(dst: torch.Tensor, src: torch.Tensor) -> None:
        """dst <- src (dtype cast) on the stream that may still be writing src (the dW side
        stream), else on the current stream."""
        side = dw_stream_for(src)
        if side is None:
            dst.copy_(src)
            return
        side.wait_stream(torch.cuda.current_stream(src.device))
        with torch.cuda.stream(side):
            dst.copy_(src)

    def launch_order(self) -> list[int]:
        """Bucket indices in the order their collectives were issued last step (tests)."""
        return list(self._issued)

    def bucket_summary(self) -> list[dict]:
        return [
            dict(bucket=b.idx, n_params=len(b.params), mb=b.flat.numel() * b.flat.element_size() / 2**20,
                 wire=str(b.cflat.dtype if b.cflat is not None else b.flat.dtype).replace("torch.", ""),
                 wire_mb=(b.cflat if b.cflat is not None else b.flat).numel()
                 * (b.cflat if b.cflat is not None else b.flat).element_size() / 2**20)
            for b in self.buckets
        ]


# Reference class names (``ddp_bucketed_overlapped_sharded.py``) for drop-in users.
DDP = DDPIndividual
DDP_Bucketed = DDPBucketed
