"""Fused AdamW (adamw_t_kernel: update + bf16 shadow + bf16 Wᵀ) timed per weight shape, to find shapes
the kernel runs below the HBM rate on (byte model 32 B per parameter).

    python scripts/adamw_shapes.py [--shapes 20480x2560,2560x10240]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

SHAPES = ["12800x1600", "1600x6400", "4800x1600", "1600x1600", "10000x1600",
          "20480x2560", "2560x10240", "7680x2560", "2560x2560", "10000x2560"]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shapes", default=",".join(SHAPES))
    ap.add_argument("--copies", type=int, default=4, help="tensors of the shape per step (more bytes per timing)")
    a = ap.parse_args()
    from cs336_systems import ops
    from cs336_systems.utils.timing import do_bench

    assert ops.load_ext(), ops.load_error()
    for sh in a.shapes.split(","):
        R, C = (int(x) for x in sh.split("x"))
        ps = [torch.nn.Parameter(torch.randn(R, C, device="cuda") * 0.02) for _ in range(a.copies)]
        for p in ps:
            p.grad = torch.randn_like(p) * 1e-3
        opt = ops.FusedAdamW(ps, lr=1e-4, betas=(0.9, 0.95), eps=1e-8, weight_decay=0.01, bf16_shadows=True)
        opt.step()
        ms = do_bench(opt.step, quantiles=(0.5,))
        n = R * C * a.copies
        print(json.dumps({"shape": sh, "ms": round(ms, 4), "TBps": round(32 * n / ms / 1e9, 2)}), flush=True)
        del opt, ps
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
