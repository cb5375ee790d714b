"""CPU test of the ``best``-mode GEMM selection (cs336_systems/ops/gemm.py ``_pick``): a low free-memory
reading drops only the split-K candidates (those that carry ``partial_bytes``); "blas" always stays in
the comparison (the filter used to drop every candidate under 4 GiB free)."""

import torch

from cs336_systems.ops import gemm


def _cands():
    def blas():
        return None

    def lt():
        return None

    def splitk():
        return None

    splitk.partial_bytes = 1 << 30
    return {"blas": blas, "lt": lt, "cs336_sk": splitk}


def _run(monkeypatch, free_bytes, times):
    monkeypatch.setattr(gemm, "_BEST", {})
    monkeypatch.setattr(gemm, "_BEST_TIMES", {})
    monkeypatch.setattr(gemm, "selection_table", lambda: {})
    monkeypatch.setattr(gemm, "_multi_rank", lambda: False)
    monkeypatch.setattr(torch.cuda, "is_current_stream_capturing", lambda: False)
    monkeypatch.setattr(torch.cuda, "mem_get_info", lambda *a, **k: (free_bytes, 288 << 30))
    timed = []

    def fake_time(fn, reps=5):
        name = next(n for n, f in cands.items() if f is fn)
        timed.append(name)
        return times[name]

    monkeypatch.setattr(gemm, "_time_ms", fake_time)
    cands = _cands()
    a, b = torch.empty(256, 64), torch.empty(64, 64)
    pick = gemm._pick("fwd", a, b, None, cands)
    return pick, timed


def test_low_free_memory_keeps_blas(monkeypatch):
    pick, timed = _run(monkeypatch, 1 << 30, {"blas": 1.0, "lt": 0.5, "cs336_sk": 0.1})
    assert "blas" in timed and "lt" in timed and "cs336_sk" not in timed
    assert pick == "lt"


def test_ample_free_memory_times_split_k(monkeypatch):
    pick, timed = _run(monkeypatch, 64 << 30, {"blas": 1.0, "lt": 0.5, "cs336_sk": 0.1})
    assert set(timed) == {"blas", "lt", "cs336_sk"}
    assert pick == "cs336_sk"


def test_near_tie_prefers_blas(monkeypatch):
    pick, _ = _run(monkeypatch, 1 << 30, {"blas": 1.0, "lt": 0.99, "cs336_sk": 0.1})
    assert pick == "blas"


def test_multi_rank_replaces_hipblaslt_table_pick(monkeypatch):
    """A committed "lt" / "blas" pick becomes the cs336 kernel in a multi-rank job (stream-K beside RCCL)."""
    monkeypatch.setattr(gemm, "_BEST", {})
    monkeypatch.setattr(gemm, "_BEST_TIMES", {})
    a, b = torch.empty(256, 64), torch.empty(64, 64)
    key = ("nt", tuple(a.shape), a.stride(), tuple(b.shape), b.stride(), None)
    monkeypatch.setattr(gemm, "selection_table", lambda: {str(key): "lt"})
    cands = {"blas": lambda: None, "lt": lambda: None, "g8": lambda: None}
    monkeypatch.setattr(gemm, "_multi_rank", lambda: True)
    assert gemm._pick("nt", a, b, None, cands) == "g8"
    monkeypatch.setattr(gemm, "_BEST", {})
    monkeypatch.setattr(gemm, "_multi_rank", lambda: False)
    assert gemm._pick("nt", a, b, None, cands) == "lt"
    # an untimed multi-rank miss: the cs336 kernel too
    monkeypatch.setattr(gemm, "_BEST", {})
    monkeypatch.setattr(gemm, "selection_table", lambda: {})
    monkeypatch.setattr(gemm, "_multi_rank", lambda: True)
    monkeypatch.setattr(torch.cuda, "is_current_stream_capturing", lambda: False)
    assert gemm._pick("nt", a, b, None, {"blas": lambda: None, "cs336": lambda: None}) == "cs336"


def test_committed_table_has_no_hipblaslt_pick_for_xl_and_2p7b():
    """The XL (52,224-token) and 2.7b (32,768-token) training steps run no hipBLASLt GEMM: every
    committed pick for their projection problems is a cs336 kernel (gemm8 or a split-K plan), so one
    GPU and multi-rank runs take the same kernels (profiles/r6_gemm_2p7b_g8.md)."""
    import json
    import os

    doc = json.load(open(gemm.TABLE_FILE))
    picks = {k: v for k, v in doc["entries"].items() if "(52224, " in k or "(32768, " in k}
    assert picks
    assert not {k: v for k, v in picks.items() if v in ("lt", "blas")}, "hipBLASLt pick in a training-step problem"
    assert os.path.basename(gemm.TABLE_FILE) == "gemm_table_mi355x.json"
