"""FlashAttention-2 adapter tests (reference ``tests/test_attention.py``), plus causal and bf16
coverage of the PyTorch path that the reference never exercised."""

import pytest
import torch
from einops import einsum

from .adapters import get_flashattention_autograd_function_pytorch, get_flashattention_autograd_function_triton


def _attention_and_lse(q, k, v, is_causal=False):
    n_queries = q.shape[-2]
    n_keys = k.shape[-2]
    d = q.shape[-1]
    scale = 1 / (d**0.5)
    S = einsum(q, k, "... q d, ... k d -> ... q k") * scale
    if is_causal:
        S = torch.where(
            torch.arange(n_queries, device=S.device)[None, :, None] >= torch.arange(n_keys, device=S.device)[None, None, :],
            S,
            -1e6,
        )
    P = torch.softmax(S, dim=-1)
    o = einsum(P, v, "... q k, ... k d -> ... q d")
    L = torch.logsumexp(S, dim=-1)
    return o, L


def _make_attn_inputs(device=None, dtype=torch.float32, B=4, N=128, D=64):
    torch.random.manual_seed(0)
    q = torch.randn(B, N, D, device=device, dtype=dtype, requires_grad=True)
    k = torch.randn(B, N, D, device=device, dtype=dtype, requires_grad=True)
    v = torch.randn(B, N, D, device=device, dtype=dtype, requires_grad=True)
    do = torch.randn(B, N, D, device=device, dtype=dtype)
    return q, k, v, do


def _test_flash_forward_pass(impl, device="cpu", is_causal=False):
    q, k, v, _do = _make_attn_inputs(device)
    o = impl(q, k, v, is_causal)
    assert o.grad_fn.saved_tensors is not None
    maybe_ls = [t for t in o.grad_fn.saved_tensors if t.shape == (q.shape[0], q.shape[1])]
    assert len(maybe_ls) == 1, f"expected exactly one saved (B, Nq) tensor, found {len(maybe_ls)}"
    l = maybe_ls[0]
    o_ref, l_ref = _attention_and_lse(q, k, v, is_causal)
    torch.testing.assert_close(o, o_ref, rtol=1e-2, atol=1e-2)
    torch.testing.assert_close(l, l_ref, rtol=1e-2, atol=1e-2)


def test_flash_forward_pass_pytorch():
    _test_flash_forward_pass(get_flashattention_autograd_function_pytorch().apply)


def test_flash_forward_pass_pytorch_causal():
    _test_flash_forward_pass(get_flashattention_autograd_function_pytorch().apply, is_causal=True)


@pytest.mark.gpu
@pytest.mark.parametrize("is_causal", [False, True])
def test_flash_forward_pass_triton(is_causal):
    _test_flash_forward_pass(get_flashattention_autograd_function_triton().apply, device="cuda", is_causal=is_causal)


def flash_backward_results(impl, is_causal, device=None):
    q, k, v, do = _make_attn_inputs(device=device)
    impl(q, k, v, is_causal).backward(do)
    return q.grad, k.grad, v.grad


@pytest.mark.parametrize("is_causal", [False, True])
def test_flash_backward_pytorch(is_causal):
    dq_e, dk_e, dv_e = flash_backward_results(lambda *a: _attention_and_lse(*a)[0], is_causal)
    q, k, v, do = _make_attn_inputs()
    get_flashattention_autograd_function_pytorch().apply(q, k, v, is_causal).backward(do)
    torch.testing.assert_close(dq_e, q.grad, rtol=1e-2, atol=1e-2)
    torch.testing.assert_close(dk_e, k.grad, rtol=1e-2, atol=1e-2)
    torch.testing.assert_close(dv_e, v.grad, rtol=1e-2, atol=1e-2)


def test_flash_pytorch_bf16_runs():
    q, k, v, do = _make_attn_inputs(dtype=torch.bfloat16, B=2, N=64, D=32)
    o = get_flashattention_autograd_function_pytorch().apply(q, k, v, True)
    assert o.dtype == torch.bfloat16
    o_ref, _ = _attention_and_lse(q.float(), k.float(), v.float(), True)
    torch.testing.assert_close(o.float(), o_ref, rtol=3e-2, atol=3e-2)
    o.backward(do)
    assert q.grad.dtype == torch.bfloat16


@pytest.mark.gpu
@pytest.mark.parametrize("is_causal", [False, True])
def test_flash_backward_triton(is_causal):
    dq_e, dk_e, dv_e = flash_backward_results(lambda *a: _attention_and_lse(*a)[0], is_causal, device="cuda")
    q, k, v, do = _make_attn_inputs(device="cuda")
    get_flashattention_autograd_function_triton().apply(q, k, v, is_causal).backward(do)
    torch.testing.assert_close(dq_e, q.grad, rtol=1e-2, atol=1e-2)
    torch.testing.assert_close(dk_e, k.grad, rtol=1e-2, atol=1e-2)
    torch.testing.assert_close(dv_e, v.grad, rtol=1e-2, atol=1e-2)
