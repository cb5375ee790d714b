"""One training step of a shallow model with a registry size's layer shape, synchronizing and
printing after every phase (for locating slow or stuck kernels).

    python scripts/debug_step.py --size 2.7b --layers 2 --ctx 1024 --batch 2
"""

import argparse
import sys
import time

import torch

sys.path.insert(0, __file__.rsplit("/scripts/", 1)[0])
from cs336_systems import ops  # noqa: E402
from cs336_systems.models import BasicsTransformerLM, get_model_config  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--size", default="2.7b")
ap.add_argument("--layers", type=int, default=2)
ap.add_argument("--ctx", type=int, default=1024)
ap.add_argument("--batch", type=int, default=2)
ap.add_argument("--trace-bwd", action="store_true", help="sync + print after every module's backward")
a = ap.parse_args()
cfg = dict(get_model_config(a.size))
cfg["num_layers"] = a.layers
dev = torch.device("cuda", 0)
t0 = time.time()


def mark(s):
    torch.cuda.synchronize()
    print(f"[{time.time() - t0:7.2f}s] {s}", flush=True)


model = BasicsTransformerLM(vocab_size=10000, context_length=a.ctx, device=dev, **cfg)
opt = ops.FusedAdamW(model.parameters(), lr=1e-4, bf16_shadows=True)
if a.trace_bwd:
    for name, m in model.named_modules():
        if name:
            m.register_full_backward_hook(lambda mod, gi, go, name=name: mark(f"  bwd done: {name}"))
mark(f"built {cfg}")
x = torch.randint(0, 10000, (a.batch, a.ctx), device=dev)
for it in range(2):
    opt.zero_grad(set_to_none=True)
    with torch.autocast("cuda", dtype=torch.bfloat16):
        logits = model(x)
        mark("forward")
        loss = ops.cross_entropy(logits, x)
    mark(f"loss {loss.item():.4f}")
    loss.backward()
    mark("backward")
    opt.step()
    mark("step")
