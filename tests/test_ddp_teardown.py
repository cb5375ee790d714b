"""A dropped DDP wrapper must not keep its model alive (bench sweep leak, round 5): every variant's
``remove_hooks`` unregisters the gradient hooks, which live in the parameters and hold the wrapper.
Runs ``sweep_variants`` (cs336_systems/bench/ddp.py) on a gloo world of one with a tiny model and
checks with weak references that no model survives it."""

import gc
import os
import weakref

import torch
import torch.distributed as dist

import cs336_systems.bench.ddp as bench_ddp
from cs336_systems.models.transformer import BasicsTransformerLM
from cs336_systems.parallel.comm import _ephemeral_low, find_free_port


def test_find_free_port_is_outside_the_ephemeral_range():
    """Rendezvous ports come from below the kernel's ephemeral range, so no outgoing connection can
    take one between the probe and the store's bind (an EADDRINUSE seen in the GPU suite)."""
    import socket

    lo = _ephemeral_low()
    for _ in range(8):
        port = find_free_port()
        if lo > 12000:
            assert 10000 <= port < lo
        with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
            s.bind(("127.0.0.1", port))


def test_sweep_frees_every_model(monkeypatch):
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ["MASTER_PORT"] = str(find_free_port())
    dist.init_process_group("gloo", rank=0, world_size=1)
    try:
        refs = []

        def tiny(name, ctx, vocab_size=100, device=None):
            m = BasicsTransformerLM(vocab_size=vocab_size, context_length=ctx, d_model=64, num_layers=2, num_heads=4,
                                    d_ff=160, device=device)
            refs.append(weakref.ref(m))
            return m

        monkeypatch.setattr(bench_ddp, "build_model", tiny)
        out = bench_ddp.sweep_variants("tiny", 32, 2, torch.device("cpu"), vocab=100, budget_s=1e9)
        gc.collect()
        assert len(refs) == len(bench_ddp.SWEEP_VARIANTS) + 2
        assert all("ms_per_step" in r for r in out["variants"]), out["variants"]
        assert sum(r() is not None for r in refs) == 0
    finally:
        dist.destroy_process_group()
