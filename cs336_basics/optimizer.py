"""AdamW + cosine LR schedule (reference ``cs336-basics/cs336_basics/optimizer.py``).

``AdamW`` here is the reference algorithm; on GPU parameters it runs the fused multi-tensor HIP
kernel (one launch per step, ``csrc/ops/adamw.hip``) and on CPU the per-tensor eager update with
the identical update order. ``ReferenceAdamW`` is the literal per-parameter Python loop, kept as
the numerics oracle for tests and the A/B benchmark.
"""

from __future__ import annotations

import math
from collections.abc import Callable, Iterable

import torch

from cs336_systems.ops.adamw import FusedAdamW


def get_cosine_lr(it: int, max_learning_rate: float, min_learning_rate: float, warmup_iters: int, cosine_cycle_iters: int):
    """Linear warmup → cosine decay → constant min LR."""
    if it < warmup_iters:
        return max_learning_rate * it / warmup_iters
    if it > cosine_cycle_iters:
        return min_learning_rate
    decay_ratio = (it - warmup_iters) / (cosine_cycle_iters - warmup_iters)
    assert 0 <= decay_ratio <= 1
    coeff = 0.5 * (1.0 + math.cos(math.pi * decay_ratio))
    return min_learning_rate + coeff * (max_learning_rate - min_learning_rate)


AdamW = FusedAdamW


class ReferenceAdamW(torch.optim.Optimizer):
    """Per-parameter Python-loop AdamW with exactly the reference math (``optimizer.py:50-86``)."""

    def __init__(self, params: Iterable[torch.nn.Parameter], lr: float = 1e-3, betas=(0.9, 0.999), eps: float = 1e-8, weight_decay: float = 0.01):
        if not 0.0 <= lr:
            raise ValueError(f"Invalid learning rate: {lr}")
        if not 0.0 <= eps:
            raise ValueError(f"Invalid epsilon value: {eps}")
        if not 0.0 <= betas[0] < 1.0:
            raise ValueError(f"Invalid beta parameter at index 0: {betas[0]}")
        if not 0.0 <= betas[1] < 1.0:
            raise ValueError(f"Invalid beta parameter at index 1: {betas[1]}")
        super().__init__(params, dict(lr=lr, betas=betas, eps=eps, weight_decay=weight_decay))

    @torch.no_grad()
    def step(self, closure: Callable | None = None):
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        for group in self.param_groups:
            for p in group["params"]:
                if p.grad is None:
                    continue
                grad = p.grad
                state = self.state[p]
                lr = group["lr"]
                b1, b2 = group["betas"]
                eps = group["eps"]
                t = state.get("t", 1)
                m = state.get("m", torch.zeros_like(grad))
                v = state.get("v", torch.zeros_like(grad))
                m = b1 * m + (1 - b1) * grad
                v = b2 * v + (1 - b2) * torch.square(grad)
                alpha_t = lr * (math.sqrt(1 - b2**t) / (1 - b1**t))
                p -= alpha_t * m / (torch.sqrt(v) + eps)
                p -= lr * group["weight_decay"] * p
                state["m"], state["v"], state["t"] = m, v, t + 1
        return loss
