"""Probe which hipBLASLt solutions exist for the XL/2.7b weight-gradient GEMMs (stream-K or not)."""
import os
import sys

import torch

sys.path.insert(0, __file__.rsplit("/scripts/", 1)[0])
os.environ.setdefault("CS336_LT_VERBOSE", "1")
from cs336_systems import ops  # noqa: E402

assert ops.load_ext(), ops.load_error()
cs = torch.ops.cs336
T = 12288
for (n_out, k_in) in [(10000, 1600), (1600, 1600), (12800, 1600), (1600, 6400), (4800, 1600)]:
    dy = torch.randn(T, n_out, device="cuda").bfloat16()
    x = torch.randn(T, k_in, device="cuda").bfloat16()
    out = torch.empty(n_out, k_in, device="cuda")
    for flags in (0, 1):
        try:
            name = cs.lt_gemm_kernel(dy, x, True, False, out, flags)
            print(n_out, k_in, flags, cs.tensile_stream_k_mode(name), name[:160], flush=True)
        except RuntimeError as e:
            print(n_out, k_in, flags, "ERROR", str(e).splitlines()[0], flush=True)
