"""Model-layer API tests on CPU: checkpoint format, generate, student API,
data loading, LR schedule, optimizer/clip semantics, and the grouped-parameter layout."""

import json
import math
import os

import numpy as np
import torch

from cs336_basics.model import BasicsTransformerLM
from cs336_basics.nn_utils import clip_gradient, cross_entropy, log_softmax, softmax
from cs336_basics.optimizer import AdamW, ReferenceAdamW, get_cosine_lr
from cs336_systems.data import get_batch, synthetic_batch
from cs336_systems.models import MODEL_CONFIGS, param_count
from cs336_systems.models.fused import grouped_view

CFG = dict(vocab_size=101, context_length=32, d_model=64, num_layers=2, num_heads=4, d_ff=96, rope_theta=10000.0)


def test_param_counts_match_handout_table():
    assert round(param_count("xl") / 1e9, 3) == 1.998
    assert round(param_count("2.7b") / 1e9, 3) == 3.407
    m = BasicsTransformerLM(**CFG)
    assert sum(p.numel() for p in m.parameters()) == (2 * 101 * 64 + 2 * (4 * 64 * 64 + 3 * 64 * 96 + 2 * 64) + 64)
    assert m.get_num_params() == sum(p.numel() for p in m.parameters()) - m.lm_head.weight.numel()
    assert set(MODEL_CONFIGS) >= {"small", "medium", "large", "xl", "2.7b"}


def test_checkpoint_roundtrip_and_orig_mod_prefix(tmp_path):
    torch.manual_seed(0)
    m = BasicsTransformerLM(**CFG)
    m.save_pretrained(str(tmp_path))
    with open(tmp_path / "model_config.json") as f:
        assert json.load(f) == CFG
    m2 = BasicsTransformerLM.from_pretrained(str(tmp_path))
    x = torch.randint(0, 101, (2, 16))
    torch.testing.assert_close(m(x), m2(x))
    sd = {"_orig_mod." + k: v for k, v in m.state_dict().items()}  # torch.compile'd checkpoint
    torch.save(sd, tmp_path / "model.pt")
    m3 = BasicsTransformerLM.from_pretrained(str(tmp_path))
    torch.testing.assert_close(m(x), m3(x))
    assert m3.layers[0].attn.q_proj.weight.untyped_storage().data_ptr() == m3.layers[0].attn.k_proj.weight.untyped_storage().data_ptr()


def test_fused_layout_is_state_dict_transparent():
    torch.manual_seed(0)
    a = BasicsTransformerLM(**CFG, fused_layout=True)
    b = BasicsTransformerLM(**CFG, fused_layout=False)
    b.load_state_dict(a.state_dict())
    assert list(a.state_dict()) == list(b.state_dict())
    w = [a.layers[1].attn.q_proj.weight, a.layers[1].attn.k_proj.weight, a.layers[1].attn.v_proj.weight]
    assert grouped_view(w) is not None
    x = torch.randint(0, 101, (2, 16))
    torch.testing.assert_close(a(x), b(x))
    a2 = a.to(torch.float64)  # _apply re-groups
    assert grouped_view([a2.layers[0].ffn.w1.weight, a2.layers[0].ffn.w3.weight]) is not None


def test_generate_topk_and_batch():
    torch.manual_seed(0)
    m = BasicsTransformerLM(**CFG)
    out = m.generate(torch.randint(0, 101, (3, 5)), max_new_tokens=4, temperature=0.7, top_k=5)
    assert out.shape == (3, 4)
    # top_k=1 is greedy
    x = torch.randint(0, 101, (1, 5))
    g = m.generate(x, max_new_tokens=3, top_k=1)
    seq = x
    for _ in range(3):
        nxt = m(seq)[:, -1].argmax(-1, keepdim=True)
        seq = torch.cat([seq, nxt], -1)
    assert torch.equal(g, seq[:, 5:])


def test_student_transformer_api():
    from cs336_basics.transformer import TransformerLM

    m = TransformerLM(d_model=64, num_heads=4, d_ff=96, vocab_size=101, context_length=32, num_layers=2, max_seq_len=64, theta=10000.0)
    assert "layers.1.ln1.weight" in m.state_dict()
    assert m(torch.randint(0, 101, (2, 48))).shape == (2, 48, 101)


def test_get_batch_and_synthetic():
    data = np.arange(1000, dtype=np.uint16)
    x, y = get_batch(data, 4, 16, "cpu")
    assert x.shape == (4, 16) and x.dtype == torch.int64
    assert torch.equal(y, x + 1)
    xs, ys = synthetic_batch(3, 8, 50, "cpu")
    assert xs.shape == ys.shape == (3, 8) and int(xs.max()) < 50


def test_cosine_lr_schedule():
    assert get_cosine_lr(0, 1.0, 0.1, 10, 100) == 0.0
    assert get_cosine_lr(5, 1.0, 0.1, 10, 100) == 0.5
    assert math.isclose(get_cosine_lr(10, 1.0, 0.1, 10, 100), 1.0)
    assert math.isclose(get_cosine_lr(55, 1.0, 0.1, 10, 100), 0.55)
    assert get_cosine_lr(101, 1.0, 0.1, 10, 100) == 0.1


def test_nn_utils_match_torch():
    x = torch.randn(5, 7)
    torch.testing.assert_close(softmax(x), torch.softmax(x, -1))
    torch.testing.assert_close(log_softmax(x), torch.log_softmax(x, -1))
    t = torch.randint(0, 7, (5,))
    torch.testing.assert_close(cross_entropy(x, t), torch.nn.functional.cross_entropy(x, t))


def test_clip_gradient_rule():
    ps = [torch.nn.Parameter(torch.randn(10)) for _ in range(3)]
    for p in ps:
        p.grad = torch.randn(10) * 10
    g0 = [p.grad.clone() for p in ps]
    n = torch.sqrt(sum((g**2).sum() for g in g0))
    clip_gradient(ps, 1.0)
    for p, g in zip(ps, g0):
        torch.testing.assert_close(p.grad, g * (1.0 / (n + 1e-6)))


def test_adamw_fused_cpu_path_equals_reference_loop():
    torch.manual_seed(0)
    p1 = [torch.nn.Parameter(torch.randn(17, 3)) for _ in range(2)]
    p2 = [torch.nn.Parameter(p.detach().clone()) for p in p1]
    o1, o2 = AdamW(p1, lr=1e-2, weight_decay=0.1), ReferenceAdamW(p2, lr=1e-2, weight_decay=0.1)
    for _ in range(4):
        for a, b in zip(p1, p2):
            g = torch.randn_like(a)
            a.grad, b.grad = g.clone(), g.clone()
        o1.step()
        o2.step()
    for a, b in zip(p1, p2):
        torch.testing.assert_close(a, b, rtol=1e-6, atol=1e-7)


def test_memory_snapshot_helper_is_noop_without_gpu(tmp_path):
    from cs336_systems.utils.memory import record_memory_history

    with record_memory_history(str(tmp_path / "x.pickle")):
        pass
    assert not os.path.exists(tmp_path / "x.pickle") or torch.cuda.is_available()
