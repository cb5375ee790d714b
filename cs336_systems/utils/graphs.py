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
