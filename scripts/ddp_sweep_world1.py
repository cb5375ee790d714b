"""Time bench.py's multi-rank DDP-variant sweep (cs336_systems/bench/ddp.py ``sweep_variants``) on ONE GPU
under an RCCL world-1 process group, at the headline model: per variant the wall time (model build,
broadcast, warmup + timed steps) and ms/step, so the sweep's budget at W = 8 can be sized from it
(VERDICT r4 item 5). Prints one JSON line.

    python scripts/ddp_sweep_world1.py [--model xl] [--ctx 512] [--batch 4]
"""

import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="xl")
    ap.add_argument("--ctx", type=int, default=512)
    ap.add_argument("--batch", type=int, default=4)
    ap.add_argument("--only-bucket", type=float, default=None, help="run only the bucketed variant at this cap (MB)")
    a = ap.parse_args()
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29611")
    os.environ["CS336_GEMM"] = "hip"  # as bench.py runs the sweep
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
    from cs336_systems.bench.ddp import sweep_variants

    t0 = time.perf_counter()
    kw = {}
    if a.only_bucket is not None:
        kw = dict(variants=(("bucketed", a.only_bucket),), zero1=False)
    out = sweep_variants(a.model, a.ctx, a.batch, dev, budget_s=1e9, **kw)
    out["total_wall_s"] = round(time.perf_counter() - t0, 2)
    print(json.dumps(out), flush=True)
    dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
