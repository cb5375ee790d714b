"""Dump (or compare) the HIP FA backward's dq/dk/dv on fixed inputs, to check two builds bitwise:
    CS336_LIB=.../variants/base/libcs336_hip.so python scripts/fa_bwd_bitwise.py dump /tmp/a.pt
    python scripts/fa_bwd_bitwise.py check /tmp/a.pt
Shapes: the low-parallelism (split) regime, with and without the mask, RoPE and positions."""

import os
import sys

import torch

os.environ.setdefault("CS336_FA_BWD", "0")  # the two-kernel form everywhere (the d 80 default uses dQ atomics: not bitwise)

from cs336_systems.models import RotaryEmbedding
from cs336_systems.ops._ext import ops as hip_ops

SHAPES = [(1, 1, 256, 32), (1, 1, 512, 16), (1, 1, 2048, 64), (1, 1, 4096, 128), (2, 3, 1000, 64), (1, 2, 2048, 80)]


def run():
    hip = hip_ops()
    out = {}
    for B, H, N, D in SHAPES:
        for causal in (True, False):
            for rope in (False, True):
                if rope and D not in (64, 128):
                    continue
                g = torch.Generator(device="cuda").manual_seed(B * 7 + N + D)
                q, k, v, do = (torch.randn(B, H, N, D, device="cuda", dtype=torch.bfloat16, generator=g) for _ in range(4))
                ra = ()
                if rope:
                    re = RotaryEmbedding(N, D, 10000.0).to("cuda")
                    ra = (re.cos.contiguous(), re.sin.contiguous(), None)
                o, lse = hip.fa_fwd(q, k, v, causal, D**-0.5, *ra)
                out[f"{B}x{H}x{N}x{D} c{int(causal)} r{int(rope)}"] = [t.cpu() for t in hip.fa_bwd(do, q, k, v, o, lse, causal, D**-0.5, *ra)]
    return out


if __name__ == "__main__":
    mode, path = sys.argv[1], sys.argv[2]
    res = run()
    if mode == "dump":
        torch.save(res, path)
        print(f"dumped {len(res)} cases")
    else:
        ref = torch.load(path, weights_only=True)
        bad = 0
        for key, grads in res.items():
            for name, a, b in zip(("dq", "dk", "dv"), grads, ref[key]):
                same = torch.equal(a.view(torch.int16), b.view(torch.int16))
                bad += not same
                if not same:
                    print(f"{key} {name}: max |diff| {(a.float() - b.float()).abs().max().item():.3g}")
        print(f"{len(res)} cases, {bad} differing tensors")
        print("BITWISE " + ("OK" if not bad else "DIFF"))
