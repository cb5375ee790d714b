"""softmax / log_softmax / cross_entropy / clip_gradient (reference ``nn_utils.py:4-30``).

``cross_entropy`` and ``clip_gradient`` dispatch to the fused HIP kernels for GPU tensors
(``csrc/ops/xent.hip``, ``csrc/ops/multi_tensor.hip``) and run the reference math on CPU.
"""

import torch

from cs336_systems import ops as _ops


def softmax(x, dim=-1):
    rescaled = x - torch.max(x, dim=dim, keepdim=True)[0]
    e = torch.exp(rescaled)
    return e / torch.sum(e, dim=dim, keepdim=True)


def log_softmax(x, dim=-1):
    x_max = torch.max(x, dim=dim, keepdim=True)[0]
    x = x - x_max
    return x - torch.log(torch.sum(torch.exp(x), dim=dim, keepdim=True))


def cross_entropy(inputs, targets):
    return _ops.cross_entropy(inputs, targets)


def clip_gradient(parameters, max_norm):
    """Global-norm clip in place; returns the pre-clip norm (device tensor, no host sync)."""
    return _ops.clip_grad_norm_(list(parameters), max_norm)
