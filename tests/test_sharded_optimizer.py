"""ZeRO-1 sharded optimizer (reference ``tests/test_sharded_optimizer.py``): bit-exact vs the
unsharded optimizer (numpy default rtol 1e-7), 2 and 3 Gloo ranks (3 ranks with the toy models
leaves one rank with few/no params — the reference crashed there)."""

from copy import deepcopy
from typing import Type

import numpy
import pytest
import torch

from cs336_basics.optimizer import AdamW as Cs336AdamW

from .adapters import get_sharded_optimizer
from .common import ToyModel, ToyModelWithTiedWeights, _cleanup_process_group, _setup_process_group, spawn


@pytest.mark.parametrize("model_class", [ToyModel, ToyModelWithTiedWeights])
@pytest.mark.parametrize("world_size", [2, 3])
def test_sharded_optimizer(model_class, world_size):
    spawn(_test_sharded_optimizer, world_size, model_class, torch.optim.AdamW)


def test_sharded_optimizer_cs336_adamw():
    spawn(_test_sharded_optimizer, 2, ToyModel, Cs336AdamW)


def _test_sharded_optimizer(rank: int, world_size: int, model_class: Type[torch.nn.Module], optimizer_cls):
    device = _setup_process_group(rank=rank, world_size=world_size, backend="gloo")
    torch.manual_seed(42)
    non_sharded_model = model_class().to(device)
    kw = dict(lr=0.1, weight_decay=0.1, betas=(0.9, 0.999), eps=1e-8)
    non_sharded_optimizer = optimizer_cls(non_sharded_model.parameters(), **kw)
    sharded_model = deepcopy(non_sharded_model)
    sharded_optimizer = get_sharded_optimizer(sharded_model.parameters(), optimizer_cls, **kw)
    for _ in range(10):
        non_sharded_optimizer.zero_grad()
        sharded_optimizer.zero_grad()
        input_ = torch.rand((32, 10)).to(device)
        labels = torch.rand((32, 5)).to(device)
        ((labels - non_sharded_model(deepcopy(input_))) ** 2).sum().backward()
        ((labels - sharded_model(deepcopy(input_))) ** 2).sum().backward()
        non_sharded_optimizer.step()
        sharded_optimizer.step()
    for a, b in zip(non_sharded_model.parameters(), sharded_model.parameters()):
        numpy.testing.assert_allclose(a.detach().cpu().numpy(), b.detach().cpu().numpy())
    _cleanup_process_group()
