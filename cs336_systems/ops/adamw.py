"""Fused multi-tensor AdamW (``csrc/ops/adamw.hip``) with the exact update order of the cs336
AdamW (``cs336-basics/cs336_basics/optimizer.py:50-86``):

    m = b1*m + (1-b1)*g ;  v = b2*v + (1-b2)*g^2
    alpha_t = lr * sqrt(1-b2^t) / (1-b1^t)
    p -= alpha_t * m / (sqrt(v) + eps)
    p -= lr * wd * p                      # decoupled decay, applied to the *updated* p

The reference runs ~9 eager kernels per parameter tensor from a Python loop (80-120 ms per step
for 3.4 B params on H100). Here the whole model is one launch per (dtype, step)
group: a chunk table (tensor pointer, chunk offset) is built on the host and every workgroup
streams one 16 KiB-per-wave chunk with 16-byte vector loads, so the step is HBM-bound
(28 B/param: read p,g,m,v; write p,m,v).

**Optimizer step overlapped with backward** (``overlap_backward=True``, GPU only). A parameter's
update needs nothing but its own final gradient, and AdamW is HBM-bound while backward is
MFMA-bound, so the update of the last layers runs on a second HIP stream while backward still
computes the gradients of the first ones. Parameters are handed over as soon as their gradient is
final: single process — from ``post_accumulate_grad`` hooks, in chunks of ~256 MB of fp32 params
(few launches, each long enough to stream at full bandwidth); with
:class:`~cs336_systems.parallel.DDPBucketed` (``ddp=``) — per bucket, right after its all-reduce is
issued, the optimizer stream waiting on that collective (``Work.wait()`` on the optimizer stream,
the host never blocks). Each hand-over also waits for the main stream and the weight-gradient side
stream (``models/fused.py``); ``step()`` updates what was not handed over and makes the main
stream wait for the optimizer stream, so the next forward reads updated weights and bf16 shadows.
Requirements: one backward per step, no gradient transform between backward and ``step()``
(clipping — the drivers enable the overlap only when ``clip == 0``), the learning rate set before
backward. The update math is unchanged, so results are bitwise identical to the plain step
(``tests/test_opt_overlap_gpu.py``).
"""

from __future__ import annotations

import math
from collections.abc import Callable, Iterable

import torch

from ._ext import ops, use_hip


def adamw_ref_(p, g, m, v, lr, beta1, beta2, eps, wd, t):
    """In-place reference update for one tensor (fp32 math)."""
    m.mul_(beta1).add_(g, alpha=1 - beta1)
    v.mul_(beta2).addcmul_(g, g, value=1 - beta2)
    alpha_t = lr * math.sqrt(1 - beta2**t) / (1 - beta1**t)
    p.sub_(alpha_t * m / (torch.sqrt(v) + eps))
    p.sub_(lr * wd * p)


def _wt_ok(p: torch.Tensor, state: dict, wt: torch.Tensor) -> bool:
    """adamw_step_t's layout contract (csrc/bindings.cpp): contiguous 2-D fp32 tensors, R and C
    multiples of 8, 16-B aligned pointers, Wᵀ a (C, R) view with unit column stride."""
    from ..models.fused import get_shadow

    g = p.grad

    def al(t):
        return t.data_ptr() % 16 == 0

    return (
        p.dim() == 2
        and p.dtype == torch.float32
        and p.shape[0] % 8 == 0
        and p.shape[1] % 8 == 0
        and p.is_contiguous()
        and g.is_contiguous()
        and wt.shape == (p.shape[1], p.shape[0])
        and wt.stride(1) == 1
        and wt.stride(0) % 8 == 0
        and al(p) and al(g) and al(state["m"]) and al(state["v"]) and al(wt) and al(get_shadow(p))
    )


class _Overlap:
    """Bookkeeping of the backward-overlapped update (see the module docstring)."""

    def __init__(self, device: torch.device, chunk_numel: int):
        self.stream = torch.cuda.Stream(device=device)
        self.chunk_numel = chunk_numel
        self.pending: list[torch.nn.Parameter] = []
        self.pending_numel = 0
        self.stepped: set[int] = set()
        self.used = False
        self.active = True
        self.hooks: list = []


class FusedAdamW(torch.optim.Optimizer):
    """Drop-in for ``cs336_basics.optimizer.AdamW`` that runs one HIP launch per step.

    State per parameter: ``m``, ``v`` (same dtype as the parameter) and ``t`` (next step index,
    starting at 1), identical to the reference so state dicts interchange.
    """

    def __init__(
        self,
        params: Iterable[torch.nn.Parameter],
        lr: float = 1e-3,
        betas: tuple[float, float] = (0.9, 0.999),
        eps: float = 1e-8,
        weight_decay: float = 0.01,
        bf16_shadows: bool = False,
        overlap_backward: bool = False,
        ddp=None,
    ):
        """``bf16_shadows=True``: every 2-D fp32 GPU weight gets a bf16 copy that the update kernel
        rewrites in the same pass; the model's GEMMs read it instead of re-casting under autocast
        (``cs336_systems/models/fused.py``)."""
        if not 0.0 <= lr:
            raise ValueError(f"Invalid learning rate: {lr}")
        if not 0.0 <= eps:
            raise ValueError(f"Invalid epsilon value: {eps}")
        if not 0.0 <= betas[0] < 1.0:
            raise ValueError(f"Invalid beta parameter at index 0: {betas[0]}")
        if not 0.0 <= betas[1] < 1.0:
            raise ValueError(f"Invalid beta parameter at index 1: {betas[1]}")
        super().__init__(params, dict(lr=lr, betas=betas, eps=eps, weight_decay=weight_decay))
        if bf16_shadows:
            from ..models.fused import attach_bf16_shadows

            attach_bf16_shadows([p for g in self.param_groups for p in g["params"]])
        self._ov: _Overlap | None = None
        # device-resident step counter per param group (enable_device_step): {id(group): (t, alpha)}
        self._dev_step: dict[int, tuple[torch.Tensor, torch.Tensor]] = {}
        self._dev_step_pending: set[int] = set()
        if overlap_backward:
            self.enable_backward_overlap(ddp=ddp)

    # ------------------------------------------------------------------------------------------
    # device-side step counter (HIP-graph capture of the whole step)
    # ------------------------------------------------------------------------------------------
    def enable_device_step(self) -> None:
        """Read the bias-corrected step size from device memory instead of a host scalar, so that a
        HIP graph that captured ``step()`` (``utils/graphs.py`` GraphedTrainStep) replays the correct
        update on every later step: the first update launch of each step is preceded by one tiny
        kernel that advances a device step counter and writes ``lr * sqrt(1 - b2^t) / (1 - b1^t)``
        (double math rounded to fp32, as the host computes it), which the update kernels read. The
        optimizer state must exist (one eager step) and every parameter of a group must be at the
        same step. ``lr`` and the betas are read at capture time; the host's per-parameter ``t``
        follows with :meth:`advance_host_step` after each replay."""
        for group in self.param_groups:
            ts = {self.state[p]["t"] for p in group["params"] if "t" in self.state[p]}
            if not ts:
                raise RuntimeError("enable_device_step: run one optimizer step first (state is created lazily)")
            if len(ts) != 1:
                raise RuntimeError(f"enable_device_step: parameters of a group are at different steps {sorted(ts)}")
            dev = group["params"][0].device
            t0 = ts.pop() - 1  # the last completed step; the step kernel advances it before use
            self._dev_step[id(group)] = (torch.full((1,), t0, dtype=torch.int64, device=dev),
                                         torch.zeros(1, dtype=torch.float32, device=dev))
        self._dev_step_pending = set(self._dev_step)

    def advance_host_step(self) -> None:
        """Host bookkeeping after a replayed captured step: each parameter's ``t`` moves on by one,
        as an eager step would have moved it (state dicts and checkpoints stay exact)."""
        for group in self.param_groups:
            for p in group["params"]:
                st = self.state.get(p)
                if st and "t" in st:
                    st["t"] += 1

    def device_step_value(self) -> int | None:
        """The device step counter of the first group (tests / checkpoints), or None."""
        if not self._dev_step:
            return None
        return int(next(iter(self._dev_step.values()))[0].item())

    # ------------------------------------------------------------------------------------------
    # update launches
    # ------------------------------------------------------------------------------------------
    def _update(self, items: list[tuple[dict, torch.nn.Parameter]]) -> None:
        """Update ``(group, param)`` pairs whose ``.grad`` is set, on the current stream.

        Weights with a transposed bf16 shadow (``models/fused.py``) go through ``adamw_step_t``,
        which also writes Wᵀ in the same pass (+2 B/param instead of a 4 B/param transpose of every
        weight in the next forward); the rest through the 1-D ``adamw_step``."""
        from ..models.fused import get_shadow, get_shadow_t, mark_shadow_synced, mark_shadow_t_synced

        # bucket by (group, device, dtype, t, shadow, Wᵀ) so each launch has one set of
        # hyper-parameters, one bias correction and all-or-nothing shadow lists
        buckets: dict[tuple, tuple[dict, list, list, list, list, list, list]] = {}
        for group, p in items:
            if p.grad.is_sparse:
                raise RuntimeError("AdamW does not support sparse gradients")
            state = self.state[p]
            if "m" not in state:
                state["m"] = torch.zeros_like(p, memory_format=torch.preserve_format)
                state["v"] = torch.zeros_like(p, memory_format=torch.preserve_format)
                state["t"] = 1
            sh = get_shadow(p)
            wt = get_shadow_t(p) if sh is not None else None
            if wt is not None and not _wt_ok(p, state, wt):
                wt = None
            key = (id(group), p.device, p.dtype, p.grad.dtype, state["t"], sh is not None, wt is not None)
            b = buckets.setdefault(key, (group, [], [], [], [], [], []))
            b[1].append(p)
            b[2].append(p.grad)
            b[3].append(state["m"])
            b[4].append(state["v"])
            if sh is not None:
                b[5].append(sh)
            if wt is not None:
                b[6].append(wt)
            state["t"] += 1
        for key, (group, ps, gs, ms, vs, ss, wts) in buckets.items():
            t = key[4]
            lr, (beta1, beta2), eps, wd = group["lr"], group["betas"], group["eps"], group["weight_decay"]
            hip = use_hip(ps[0]) and all(x.is_contiguous() for x in ps + gs + ms + vs + ss)
            alpha = None
            if id(group) in self._dev_step:
                if not hip:
                    raise RuntimeError("enable_device_step needs the HIP update kernels")
                tdev, alpha = self._dev_step[id(group)]
                if id(group) in self._dev_step_pending:  # first update launch of this step
                    ops().adamw_device_step(tdev, alpha, lr, beta1, beta2)
                    self._dev_step_pending.discard(id(group))
            if hip and wts:
                ops().adamw_step_t(ps, gs, ms, vs, ss, wts, lr, beta1, beta2, eps, wd, t, alpha)
            elif hip:
                ops().adamw_step(ps, gs, ms, vs, ss, lr, beta1, beta2, eps, wd, t, alpha)
            else:
                for p, g, m, v in zip(ps, gs, ms, vs):
                    adamw_ref_(p, g.to(p.dtype), m, v, lr, beta1, beta2, eps, wd, t)
                for p, s in zip(ps, ss):
                    s.copy_(p)
                for p, w in zip(ps, wts):
                    w.copy_(get_shadow(p).t())
            for p in ps if ss else ():
                mark_shadow_synced(p)
            for p in ps if wts else ():
                mark_shadow_t_synced(p)

    @torch.no_grad()
    def step(self, closure: Callable | None = None):
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        ov = self._ov
        if ov is not None:
            self._flush()
        items = [
            (g, p)
            for g in self.param_groups
            for p in g["params"]
            if p.grad is not None and (ov is None or id(p) not in ov.stepped)
        ]
        if items and ov is not None and ov.used and self._dev_step:
            # the device step kernel of this step ran on the optimizer stream: the updates left for
            # this stream read its step size
            torch.cuda.current_stream(ov.stream.device).wait_stream(ov.stream)
        if items:
            self._update(items)
        if ov is not None:
            ov.stepped.clear()
            if ov.used:
                torch.cuda.current_stream(ov.stream.device).wait_stream(ov.stream)
                ov.used = False
        self._dev_step_pending = set(self._dev_step)
        return loss

    # ------------------------------------------------------------------------------------------
    # backward overlap
    # ------------------------------------------------------------------------------------------
    def enable_backward_overlap(self, ddp=None, chunk_mb: float = 256.0) -> bool:
        """Start updating parameters during backward (module docstring). Returns False (and stays
        off) when it cannot apply: CPU parameters, or a DDP wrapper whose reduced gradients are not
        final when its collective completes (non-AVG backends divide afterwards)."""
        params = [p for g in self.param_groups for p in g["params"]]
        if not params or not all(p.is_cuda for p in params) or self._ov is not None:
            return self._ov is not None
        if ddp is not None and not (hasattr(ddp, "add_bucket_callback") and getattr(ddp, "_avg", False)):
            return False
        if ddp is not None and hasattr(ddp, "supports_bucket_callbacks") and not ddp.supports_bucket_callbacks():
            return False
        ov = _Overlap(params[0].device, max(1, int(chunk_mb * 2**20 / 4)))
        self._group_of = {id(p): g for g in self.param_groups for p in g["params"]}
        if ddp is not None:
            ddp.add_bucket_callback(self._on_bucket_reduced)
        else:
            ov.hooks = [p.register_post_accumulate_grad_hook(self._on_grad_ready) for p in params if p.requires_grad]
        self._ov = ov
        return True

    def set_backward_overlap(self, active: bool) -> None:
        """Pause (e.g. for gradient-accumulation micro-steps) or resume the overlapped update."""
        if self._ov is not None:
            self._ov.active = active

    @property
    def overlaps_backward(self) -> bool:
        return self._ov is not None and self._ov.active

    def _on_grad_ready(self, p: torch.nn.Parameter) -> None:
        ov = self._ov
        # inside a HIP-graph capture only with the device-side step counter (utils/graphs.py
        # GraphedTrainStep): otherwise the update would be captured with this step's bias correction
        # and replayed on every later step as well
        if ov is None or not ov.active or p.grad is None or (torch.cuda.is_current_stream_capturing() and not self._dev_step):
            return
        ov.pending.append(p)
        ov.pending_numel += p.numel()
        if ov.pending_numel >= ov.chunk_numel:
            self._flush()

    def _on_bucket_reduced(self, params, work) -> None:
        ov = self._ov
        if ov is None or not ov.active or (torch.cuda.is_current_stream_capturing() and not self._dev_step):
            return
        ov.pending.extend(p for p in params if p.grad is not None)
        self._flush(work)

    @torch.no_grad()
    def _flush(self, work=None) -> None:
        ov = self._ov
        ps = ov.pending
        if not ps:
            return
        ov.pending, ov.pending_numel = [], 0
        from ..models.fused import dw_stream_for

        s = ov.stream
        s.wait_stream(torch.cuda.current_stream(s.device))
        side = dw_stream_for(ps[0].grad)  # weight-gradient GEMMs still in flight
        if side is not None:
            s.wait_stream(side)
        with torch.cuda.stream(s):
            if work is not None:
                work.wait()
            self._update([(self._group_of[id(p)], p) for p in ps])
        for p in ps:
            p.grad.record_stream(s)
            ov.stepped.add(id(p))
        ov.used = True


def multi_tensor_l2norm(tensors: list[torch.Tensor]) -> torch.Tensor:
    """Global L2 norm over a list of tensors as a 0-d fp32 device tensor (no host sync)."""
    tensors = [t for t in tensors if t is not None and t.numel() > 0]
    if not tensors:
        return torch.zeros(())
    if use_hip(tensors[0]) and all(t.is_contiguous() for t in tensors):
        return ops().multi_tensor_l2norm(tensors)
    total = torch.zeros((), dtype=torch.float32, device=tensors[0].device)
    for t in tensors:
        total = total + t.float().pow(2).sum()
    return total.sqrt()


def clip_grad_norm_(parameters: Iterable[torch.nn.Parameter], max_norm: float) -> torch.Tensor:
    """Global-norm clip with the cs336 rule ``g *= min(1, max_norm / (norm + 1e-6))``
    (``cs336-basics/cs336_basics/nn_utils.py:20-30``) fully on device: one multi-tensor norm
    kernel + one multi-tensor scale kernel, no ``.item()``."""
    grads = [p.grad for p in parameters if p.grad is not None]
    if not grads:
        return torch.zeros(())
    norm = multi_tensor_l2norm(grads)
    coef = torch.clamp(max_norm / (norm + 1e-6), max=1.0)
    if use_hip(grads[0]) and all(g.is_contiguous() for g in grads):
        ops().multi_tensor_scale_(grads, coef)
    else:
        for g in grads:
            g.mul_(coef.to(g.dtype))
    return norm
