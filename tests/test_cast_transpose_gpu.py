"""fp32 -> bf16 cast that also writes the transpose (csrc/ops/transpose.hip cast_t_kernel), the compiled
model's forward weight + saved Wᵀ when no bf16 shadows exist (models/compiled.py ``_weights``):
both outputs equal PyTorch's round-to-nearest-even cast, including a strided grouped view and shapes
that are not multiples of the 256 x 64 workgroup tile."""

import pytest
import torch

from cs336_systems.ops._ext import ops as _hip

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.mark.parametrize("R,C", [(1600, 1600), (4800, 1600), (10000, 1600), (72, 40), (256, 8), (8, 264)])
def test_cast_transpose_matches_torch(R, C):
    torch.manual_seed(R + C)
    x = torch.randn(R, C, device=DEV) * 3
    w, wt = _hip().cast_transpose_bf16(x)
    ref = x.to(torch.bfloat16)
    assert torch.equal(w, ref)
    assert torch.equal(wt, ref.t().contiguous())


def test_cast_transpose_of_row_block_view():
    big = torch.randn(3 * 640, 1600, device=DEV)
    v = big[640:1920]  # row-adjacent block (a grouped weight view)
    w, wt = _hip().cast_transpose_bf16(v)
    assert torch.equal(w, v.to(torch.bfloat16)) and torch.equal(wt, v.to(torch.bfloat16).t().contiguous())
