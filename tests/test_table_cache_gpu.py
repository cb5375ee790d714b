"""Multi-tensor launches reuse a cached device copy of their pointer table when the table repeats
(csrc/bindings.cpp ``device_table``): results must follow the tensors' current contents, tables
that differ only in one pointer must not alias, and a table built on one stream must be usable
from another stream and after the tensors it named were freed and their memory reused."""

import pytest
import torch

from cs336_systems.ops._ext import ops as _hip

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _ref_norm(ts):
    return torch.sqrt(sum((t.double() ** 2).sum() for t in ts)).item()


def test_repeated_table_follows_contents():
    hip = _hip()
    ts = [torch.randn(n, device=DEV) for n in (1000, 4096, 33)]
    for _ in range(3):  # same pointers every call: cached table, fresh data
        for t in ts:
            t.normal_()
        assert hip.multi_tensor_l2norm(ts).item() == pytest.approx(_ref_norm(ts), rel=1e-5)


def test_one_pointer_differs():
    hip = _hip()
    a = [torch.randn(4096, device=DEV) for _ in range(3)]
    b = a[:2] + [torch.randn(4096, device=DEV) * 10]
    na, nb = hip.multi_tensor_l2norm(a).item(), hip.multi_tensor_l2norm(b).item()
    assert na == pytest.approx(_ref_norm(a), rel=1e-5)
    assert nb == pytest.approx(_ref_norm(b), rel=1e-5)
    assert hip.multi_tensor_l2norm(a).item() == pytest.approx(na, rel=1e-6)


def test_other_stream_and_reused_memory():
    hip = _hip()
    ts = [torch.randn(8192, device=DEV) for _ in range(4)]
    expect = _ref_norm(ts)
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        got = hip.multi_tensor_l2norm(ts)
    torch.cuda.current_stream().wait_stream(s)
    assert got.item() == pytest.approx(expect, rel=1e-5)
    assert hip.multi_tensor_l2norm(ts).item() == pytest.approx(expect, rel=1e-5)
    del ts
    torch.cuda.synchronize()
    new = [torch.full((8192,), 2.0, device=DEV) for _ in range(4)]  # may land on the same addresses
    assert hip.multi_tensor_l2norm(new).item() == pytest.approx(_ref_norm(new), rel=1e-5)
    scale = torch.tensor([0.5], device=DEV)
    hip.multi_tensor_scale_(new, scale)
    assert all(torch.all(t == 1.0).item() for t in new)


@pytest.mark.parametrize("cached_first", [False, True])
def test_captured_launch_keeps_its_table(cached_first):
    """A multi-tensor launch captured in a HIP graph bakes in the table's device address: the table
    must stay valid (and hold the same contents) on every replay, whether it was first built inside
    the capture (its copy node re-reads the host buffer) or taken from the cache built before it, and
    no later eviction may free it (more distinct tables than the cache bound are built in between)."""
    hip = _hip()
    ts = [torch.randn(n, device=DEV) for n in (5000, 64, 777)]
    if cached_first:
        hip.multi_tensor_l2norm(ts)
        torch.cuda.synchronize()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    g = torch.cuda.CUDAGraph()
    with torch.cuda.stream(s):
        hip.multi_tensor_l2norm(ts)  # warm the capturing stream's table
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    with torch.cuda.graph(g):
        out = hip.multi_tensor_l2norm(ts)
    # churn the evictable cache past its bound with tables that never repeat
    junk = [torch.zeros(64, device=DEV) for _ in range(4200)]  # held: every table names new addresses
    for t in junk:
        hip.multi_tensor_l2norm([t])
    torch.cuda.synchronize()
    for _ in range(3):
        for t in ts:
            t.normal_()
        g.replay()
        torch.cuda.synchronize()
        assert out.item() == pytest.approx(_ref_norm(ts), rel=1e-5)
