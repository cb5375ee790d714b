"""Cross-entropy over logits (``cs336-basics/cs336_basics/nn_utils.py:9-17``): mean over rows of
``logsumexp(z) - z[target]``.

HIP path (``csrc/ops/xent.hip``): one workgroup per row computes an online max/sum-exp over the
vocab in a single read of the (bf16 or fp32) logits, writes the per-row loss and LSE; the
backward writes ``(softmax - onehot) * g / M`` in the logits dtype in one pass. The upstream
gradient ``g`` is read from device memory, so there is no host sync anywhere in the loss.
"""

from __future__ import annotations

import torch

from ._ext import ops, use_hip


def log_softmax_ref(x: torch.Tensor, dim: int = -1) -> torch.Tensor:
    x_max = torch.max(x, dim=dim, keepdim=True)[0]
    x = x - x_max
    return x - torch.log(torch.sum(torch.exp(x), dim=dim, keepdim=True))


def cross_entropy_ref(inputs: torch.Tensor, targets: torch.Tensor) -> torch.Tensor:
    nls = -log_softmax_ref(inputs.float())
    return torch.mean(torch.gather(nls, -1, targets.unsqueeze(-1)))


class CrossEntropyHIP(torch.autograd.Function):
    @staticmethod
    def forward(ctx, logits, targets):
        V = logits.shape[-1]
        z = logits.reshape(-1, V)
        if not z.is_contiguous():
            z = z.contiguous()
        t = targets.reshape(-1).to(torch.int64).contiguous()
        loss_rows, lse = ops().xent_fwd(z, t)
        ctx.save_for_backward(z, t, lse)
        ctx.shape = logits.shape
        return loss_rows.mean()

    @staticmethod
    def backward(ctx, g):
        z, t, lse = ctx.saved_tensors
        g = g.reshape(()).float().contiguous()
        dz = ops().xent_bwd(g, z, t, lse, 1.0 / z.shape[0])
        return dz.view(ctx.shape), None


def cross_entropy(logits: torch.Tensor, targets: torch.Tensor) -> torch.Tensor:
    if use_hip(logits):
        return CrossEntropyHIP.apply(logits, targets)
    return cross_entropy_ref(logits, targets)
