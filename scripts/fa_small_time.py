"""Where the B 1 H 1 small-N backward's time goes: do_bench with / without the cache flush, host
enqueue time per call, and back-to-back GPU time per call (events around 200 calls).
    FA_SMALL="1,1,256,32,1" python scripts/fa_small_time.py   (CS336_LIB=... to pick a build)"""

import json
import os
import time

import torch

from cs336_systems.ops.flash_attention import FlashAttentionHIP
from cs336_systems.utils.timing import do_bench

for sh in os.environ.get("FA_SMALL", "1,1,256,32,1;1,1,8192,32,1").split(";"):
    B, H, N, D, c = (int(x) for x in sh.split(","))
    q, k, v = (torch.randn(B, H, N, D, device="cuda", dtype=torch.bfloat16, requires_grad=True) for _ in range(3))
    o = FlashAttentionHIP.apply(q, k, v, bool(c))
    do = torch.randn_like(o)
    fn = lambda: torch.autograd.grad(o, (q, k, v), do, retain_graph=True)
    row = {"B": B, "H": H, "N": N, "D": D, "causal": c}
    row["bench_flush_us"] = round(do_bench(fn, warmup=20, rep=200)[0] * 1e3, 1)
    row["bench_noflush_us"] = round(do_bench(fn, warmup=20, rep=200, flush_cache=False)[0] * 1e3, 1)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(200):
        fn()
    row["host_enqueue_us"] = round((time.perf_counter() - t0) / 200 * 1e6, 1)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(200):
        fn()
    e1.record()
    torch.cuda.synchronize()
    row["back_to_back_us"] = round(e0.elapsed_time(e1) / 200 * 1e3, 1)
    print(json.dumps(row), flush=True)
