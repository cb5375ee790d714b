"""Bucketed DDP test (reference ``tests/test_ddp.py``): 2 Gloo ranks on CPU, toy models with a
frozen bias, a frozen parameter and tied weights; DDP must match single-process SGD exactly."""

import logging
from copy import deepcopy
from typing import Type

import pytest
import torch
import torch.distributed as dist
import torch.nn as nn
import torch.optim as optim

from .adapters import ddp_bucketed_on_after_backward, ddp_bucketed_on_train_batch_start, get_ddp_bucketed
from .common import (
    FIXTURES_PATH,
    ToyModel,
    ToyModelWithTiedWeights,
    _cleanup_process_group,
    _setup_process_group,
    spawn,
    validate_ddp_net_equivalence,
)

logger = logging.getLogger(__name__)


@pytest.mark.parametrize("model_class", [ToyModel, ToyModelWithTiedWeights])
@pytest.mark.parametrize("bucket_size_mb", [0.0016, 0.0001, 0.01, None])
def test_DistributedDataParallelCPU(bucket_size_mb, model_class):
    spawn(_test_DistributedDataParallelCPU, 2, bucket_size_mb, model_class)


def _test_DistributedDataParallelCPU(rank: int, world_size: int, bucket_size_mb: float, model_class: Type[torch.nn.Module]):
    device = _setup_process_group(rank=rank, world_size=world_size, backend="gloo")
    dist.barrier()
    torch.manual_seed(rank)
    non_parallel_model = model_class().to(device)
    ddp_base = deepcopy(non_parallel_model)
    ddp_model = get_ddp_bucketed(ddp_base, bucket_size_mb=bucket_size_mb)
    for (np_name, np_param), (ddp_name, ddp_param) in zip(non_parallel_model.named_parameters(), ddp_model.named_parameters()):
        fixed = "no_grad_fixed_param" in ddp_name or "no_grad_fixed_param" in np_name
        if rank == 0 or fixed:
            assert torch.allclose(np_param, ddp_param)
        else:
            assert not torch.allclose(np_param, ddp_param)
    validate_ddp_net_equivalence(ddp_model)
    all_x = torch.load(FIXTURES_PATH / "ddp_test_data.pt", weights_only=True)
    all_y = torch.load(FIXTURES_PATH / "ddp_test_labels.pt", weights_only=True)
    assert all_x.size(0) % world_size == 0
    local_bs = int(all_y.size(0) / world_size)
    loss_fn = nn.MSELoss()
    ddp_optimizer = optim.SGD(ddp_model.parameters(), lr=0.1)
    non_parallel_optimizer = optim.SGD(non_parallel_model.parameters(), lr=0.1)
    for i in range(5):
        ddp_bucketed_on_train_batch_start(ddp_model=ddp_model, optimizer=ddp_optimizer)
        ddp_optimizer.zero_grad()
        non_parallel_optimizer.zero_grad()
        non_parallel_loss = loss_fn(non_parallel_model(all_x.to(device)), all_y.to(device))
        non_parallel_loss.backward()
        non_parallel_optimizer.step()
        if rank == 0:
            for a, b in zip(non_parallel_model.parameters(), ddp_model.parameters()):
                if a.requires_grad and b.requires_grad:
                    assert not torch.allclose(a, b)
                else:
                    assert torch.allclose(a, b)
        offset = rank * local_bs
        ddp_loss = loss_fn(ddp_model(all_x[offset : offset + local_bs, :].to(device)), all_y[offset : offset + local_bs, :].to(device))
        ddp_loss.backward()
        ddp_bucketed_on_after_backward(ddp_model=ddp_model, optimizer=ddp_optimizer)
        ddp_optimizer.step()
        if rank == 0:
            for a, b in zip(non_parallel_model.parameters(), ddp_model.parameters()):
                assert torch.allclose(a, b)
        torch.manual_seed(42 + i)
        shuffle_idxs = torch.randperm(all_x.size(0))
        all_x = all_x[shuffle_idxs]
        all_y = all_y[shuffle_idxs]
    if rank == 0:
        for a, b in zip(non_parallel_model.parameters(), ddp_model.parameters()):
            assert torch.allclose(a, b)
    _cleanup_process_group()
