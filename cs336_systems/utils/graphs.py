"""HIP-graph capture of a training step (forward + loss + backward) for launch-bound models.

The reference measures ``torch.compile`` (an Inductor/Triton tracing compiler) against eager mode
(``cs336_systems/benchmark.py:43-44``). On MI355X the launch-bound regime — small models, short
sequences, a few thousand tokens per step, where the host issues kernels slower than the GPU
retires them — is addressed without a compiler: the whole forward + cross-entropy + backward is
recorded once into a HIP graph (``torch.cuda.CUDAGraph``, hipGraph on ROCm) and replayed with one
launch. All kernels of the step (hipBLASLt GEMMs, the cs336 HIP ops, the embedding backward)
are stream-ordered and free of host syncs, and the side-stream Wᵀ copies stay on the capturing
stream while a capture is in progress (``models/fused.py``).

Contract: inputs are copied into static buffers; gradients are written into the same (graph-pool)
tensors on every replay and re-attached to ``p.grad`` afterwards, so the optimizer runs eagerly
after :meth:`GraphedStep.__call__` (do not ``zero_grad(set_to_none=True)`` in between — the next
replay overwrites the gradients, it does not accumulate). Parameters must keep their storage
(optimizer updates are in place, as FusedAdamW's are). ``tests/test_graphs_gpu.py`` checks
replayed losses and gradients against eager steps.
"""

from __future__ import annotations

from collections.abc import Callable

import torch


class GraphedStep:
    """``loss = step(x, y)`` replays the captured forward + backward of ``loss_fn(x, y)``."""

    def __init__(self, loss_fn: Callable[[torch.Tensor, torch.Tensor], torch.Tensor], params, x: torch.Tensor, y: torch.Tensor, warmup: int = 3):
        if not x.is_cuda:
            raise ValueError("GraphedStep captures HIP graphs: inputs must be GPU tensors")
        self.params = [p for p in params if p.requires_grad]
        self.x, self.y = x.clone(), y.clone()
        dev = x.device
        # warm up on a side stream (allocator pools, hipBLASLt heuristics, lazy inits) before capture
        s = torch.cuda.Stream(device=dev)
        s.wait_stream(torch.cuda.current_stream(dev))
        with torch.cuda.stream(s):
            for _ in range(warmup):
                for p in self.params:
                    p.grad = None
                loss_fn(self.x, self.y).backward()
        torch.cuda.current_stream(dev).wait_stream(s)
        torch.cuda.synchronize(dev)
        for p in self.params:
            p.grad = None
        self.graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(self.graph):
            self.loss = loss_fn(self.x, self.y)
            self.loss.backward()
        self.grads = [p.grad for p in self.params]

    def __call__(self, x: torch.Tensor, y: torch.Tensor) -> torch.Tensor:
        self.x.copy_(x)
        self.y.copy_(y)
        self.graph.replay()
        for p, g in zip(self.params, self.grads):
            p.grad = g
        return self.loss


class GraphedTrainStep:
    """The WHOLE training step -- zero grads, forward, loss, backward and the optimizer update,
    including an update overlapped with the backward on a side stream -- captured once into one HIP
    graph and replayed with one launch per step (the eager step loses ~5 ms of
    XL step time to launch and host gaps, ``profiles/r5_opt_overlap_ab.md``).

    ``step_fn(x, y) -> loss`` must run one complete eager step on the current stream, starting with
    ``optimizer.zero_grad(set_to_none=True)`` and ending with ``optimizer.step()``. The constructor
    runs ``warmup`` such steps on the capture stream (REAL training steps: they update the weights;
    they also create the optimizer state, which must not be allocated inside the graph), switches
    the optimizer to its device-side step counter (``FusedAdamW.enable_device_step``: the bias
    correction is computed on the GPU at every replay) and captures one more step without executing
    it. Each call copies the batch into the captured input buffers, replays, and advances the
    optimizer's host-side step counters. Gradients live in the graph's memory pool and are
    rewritten by every replay; the parameters and optimizer state keep their storage (in-place
    updates). Hyper-parameters (lr, betas, weight decay) are fixed at capture time.
    ``tests/test_graphs_gpu.py`` checks a replayed run bitwise against the eager one."""

    def __init__(self, step_fn: Callable[[torch.Tensor, torch.Tensor], torch.Tensor], optimizer, x: torch.Tensor,
                 y: torch.Tensor, warmup: int = 1):
        if not x.is_cuda:
            raise ValueError("GraphedTrainStep captures HIP graphs: inputs must be GPU tensors")
        if not hasattr(optimizer, "enable_device_step"):
            raise TypeError("GraphedTrainStep needs an optimizer with a device-side step counter (FusedAdamW)")
        self.opt = optimizer
        self.x, self.y = x.clone(), y.clone()
        dev = x.device
        self.stream = torch.cuda.Stream(device=dev)
        self.stream.wait_stream(torch.cuda.current_stream(dev))
        with torch.cuda.stream(self.stream):
            for _ in range(max(1, warmup)):
                self.warmup_loss = step_fn(self.x, self.y).detach()
        torch.cuda.current_stream(dev).wait_stream(self.stream)
        torch.cuda.synchronize(dev)
        optimizer.enable_device_step()
        params = [p for g in optimizer.param_groups for p in g["params"]]
        t_host = [(p, optimizer.state[p]["t"]) for p in params if "t" in optimizer.state[p]]
        for p in params:  # the eager pool's blocks are not reusable by the graph's private pool
            p.grad = None
        torch.cuda.empty_cache()
        self.graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(self.graph, stream=self.stream):
            self.loss = step_fn(self.x, self.y)
        for p, t in t_host:  # capturing executed nothing: undo the host-side step bookkeeping
            optimizer.state[p]["t"] = t

    def __call__(self, x: torch.Tensor, y: torch.Tensor) -> torch.Tensor:
        self.x.copy_(x)
        self.y.copy_(y)
        self.graph.replay()
        self.opt.advance_host_step()
        return self.loss
