"""Time one fused AdamW step over the XL (or any) model's parameters with the bf16 / Wᵀ shadows, as
bench.py runs it (ops/adamw.py FusedAdamW, csrc/ops/multi_tensor.hip adamw_t_kernel for 2-D weights).

    python scripts/adamw_bench.py [--model xl] [--iters 20]

Prints one JSON line: ms per step and the HBM rate of the byte model (fp32 p/m/v read+write, fp32
grad read, bf16 shadow and Wᵀ writes = 32 B per parameter; 28 B for the ones without Wᵀ).
"""

import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="xl")
    ap.add_argument("--ctx", type=int, default=512)
    ap.add_argument("--iters", type=int, default=20)
    args = ap.parse_args()

    from cs336_systems import ops
    from cs336_systems.models import build_model

    assert ops.load_ext(), ops.load_error()
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    model = build_model(args.model, args.ctx, device=dev)
    opt = ops.FusedAdamW(model.parameters(), lr=1e-4, betas=(0.9, 0.95), eps=1e-8, weight_decay=0.01,
                         bf16_shadows=True)
    n = 0
    for p in model.parameters():
        p.grad = torch.randn_like(p) * 1e-3
        n += p.numel()
    for _ in range(3):
        opt.step()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(args.iters):
        opt.step()
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / args.iters
    print(json.dumps({"model": args.model, "params": n, "ms_per_step": round(ms, 3),
                      "tb_per_s_32B": round(n * 32 / ms / 1e9, 2)}))


if __name__ == "__main__":
    main()
