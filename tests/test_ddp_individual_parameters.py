"""Per-parameter overlapped DDP (reference ``tests/test_ddp_individual_parameters.py``) plus the
naive and flat variants, all against single-process training on 2 Gloo ranks."""

from copy import deepcopy
from typing import Type

import pytest
import torch
import torch.distributed as dist
import torch.nn as nn
import torch.optim as optim

from cs336_systems.parallel import FlatDDP, NaiveDDP

from .adapters import ddp_individual_parameters_on_after_backward, get_ddp_individual_parameters
from .common import (
    FIXTURES_PATH,
    ToyModel,
    ToyModelWithTiedWeights,
    _cleanup_process_group,
    _setup_process_group,
    spawn,
    validate_ddp_net_equivalence,
)

_WRAPPERS = {
    "individual": get_ddp_individual_parameters,
    "naive": NaiveDDP,
    "flat": FlatDDP,
}


@pytest.mark.parametrize("model_class", [ToyModel, ToyModelWithTiedWeights])
@pytest.mark.parametrize("variant", ["individual", "naive", "flat"])
def test_DistributedDataParallelIndividualParameters(model_class, variant):
    spawn(_test_ddp, 2, model_class, variant)


def _test_ddp(rank: int, world_size: int, model_class: Type[torch.nn.Module], variant: str):
    device = _setup_process_group(rank=rank, world_size=world_size, backend="gloo")
    dist.barrier()
    torch.manual_seed(rank)
    non_parallel_model = model_class().to(device)
    ddp_model = _WRAPPERS[variant](deepcopy(non_parallel_model))
    for (n1, p1), (n2, p2) in zip(non_parallel_model.named_parameters(), ddp_model.named_parameters()):
        fixed = "no_grad_fixed_param" in n1 or "no_grad_fixed_param" in n2
        if rank == 0 or fixed:
            assert torch.allclose(p1, p2)
        else:
            assert not torch.allclose(p1, p2)
    validate_ddp_net_equivalence(ddp_model)
    all_x = torch.load(FIXTURES_PATH / "ddp_test_data.pt", weights_only=True)
    all_y = torch.load(FIXTURES_PATH / "ddp_test_labels.pt", weights_only=True)
    local_bs = int(all_y.size(0) / world_size)
    loss_fn = nn.MSELoss()
    ddp_optimizer = optim.SGD(ddp_model.parameters(), lr=0.1)
    non_parallel_optimizer = optim.SGD(non_parallel_model.parameters(), lr=0.1)
    for i in range(5):
        ddp_optimizer.zero_grad()
        non_parallel_optimizer.zero_grad()
        loss_fn(non_parallel_model(all_x.to(device)), all_y.to(device)).backward()
        non_parallel_optimizer.step()
        offset = rank * local_bs
        loss_fn(ddp_model(all_x[offset : offset + local_bs].to(device)), all_y[offset : offset + local_bs].to(device)).backward()
        ddp_individual_parameters_on_after_backward(ddp_model, ddp_optimizer)
        ddp_optimizer.step()
        if rank == 0:
            for a, b in zip(non_parallel_model.parameters(), ddp_model.parameters()):
                assert torch.allclose(a, b)
        torch.manual_seed(42 + i)
        idx = torch.randperm(all_x.size(0))
        all_x, all_y = all_x[idx], all_y[idx]
    _cleanup_process_group()
