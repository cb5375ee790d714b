"""Where does a torch.compile'd train step spend its time? Runs e2e's step on a model size with
faulthandler stack dumps every 45 s and per-step timestamps (diagnostic for slow compiles).

    python scripts/compile_debug.py [--size small] [--steps 3]
"""
import argparse
import faulthandler
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--size", default="small")
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--batch", type=int, default=4)
    ap.add_argument("--fullgraph", action="store_true")
    a = ap.parse_args()
    faulthandler.dump_traceback_later(45, repeat=True, file=sys.stderr)
    from cs336_systems import ops
    from cs336_systems.models import build_model

    dev = torch.device("cuda", 0)
    model = build_model(a.size, 512, device=dev)
    opt = ops.FusedAdamW(model.parameters(), lr=1e-4)
    fm = torch.compile(model, fullgraph=a.fullgraph)
    x = torch.randint(0, 10000, (a.batch, 512), device=dev)
    t0 = time.time()
    for i in range(a.steps):
        opt.zero_grad(set_to_none=True)
        with torch.autocast("cuda", dtype=torch.bfloat16):
            loss = ops.cross_entropy(fm(x), x)
        print(f"step {i} fwd done {time.time() - t0:.1f}s", flush=True)
        loss.backward()
        print(f"step {i} bwd done {time.time() - t0:.1f}s", flush=True)
        opt.step()
        torch.cuda.synchronize()
        print(f"step {i} done {time.time() - t0:.1f}s loss {loss.item():.4f}", flush=True)
    faulthandler.cancel_dump_traceback_later()


if __name__ == "__main__":
    main()
