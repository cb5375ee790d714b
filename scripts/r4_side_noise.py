"""The XL training step (forward + backward, cs336 kernels) alone vs with RCCL-like work on a second
stream, on one GPU: (a) 'occupy': back-to-back RCCL-channel-shaped resident workgroups (64 x 256
threads, 21 KB LDS, 1 ms each), (b) 'copy': back-to-back 128 MB device copies (bucket-sized traffic).
Tells whether the step degrades in proportion to the CUs / bandwidth taken (expected for any
overlap) or collapses the way the dW side stream does (profiles/r4_dw_stream.md).

    python scripts/r4_side_noise.py [--batch 16]
"""
import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=16)
    ap.add_argument("--iters", type=int, default=5)
    a = ap.parse_args()
    from cs336_systems import ops
    from cs336_systems.models import build_model

    assert ops.load_ext(), ops.load_error()
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    model = build_model("xl", 512, vocab_size=10000, device=dev)
    x = torch.randint(0, 10000, (a.batch, 512), device=dev)

    def step():
        with torch.autocast("cuda", dtype=torch.bfloat16):
            loss = ops.cross_entropy(model(x), x)
        loss.backward()

    for _ in range(2):
        step()
    torch.cuda.synchronize()
    side = torch.cuda.Stream()
    counter = torch.zeros(1, dtype=torch.int32, device=dev)
    src = torch.empty(32 * 1024 * 1024, device=dev)
    dst = torch.empty_like(src)

    def timed(noise):
        stop = [False]
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(a.iters):
            if noise:
                with torch.cuda.stream(side):
                    for _ in range(40):  # enough side work to span the step
                        if noise == "occupy":
                            torch.ops.cs336.occupy(64, 21184, 1.0, counter)
                        else:
                            dst.copy_(src)
            step()
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) * 1e3 / a.iters

    res = {"batch": a.batch}
    for mode in ("alone", "occupy", "copy", "alone2"):
        res[mode + "_ms"] = round(timed(None if mode.startswith("alone") else mode), 2)
        print(json.dumps({mode: res[mode + "_ms"]}), flush=True)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
