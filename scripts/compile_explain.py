"""Graph breaks of ``torch.compile(model)`` on the HIP path: ``torch._dynamo.explain`` over one
forward (and the loss) of a model under bf16 autocast, printing the break count and every reason.

    python scripts/compile_explain.py [--size xl] [--batch 2] [--ctx 512]
"""

import argparse
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

import torch  # noqa: E402


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--size", default="xl")
    ap.add_argument("--batch", type=int, default=2)
    ap.add_argument("--ctx", type=int, default=512)
    a = ap.parse_args()
    from cs336_systems import ops
    from cs336_systems.models import build_model

    assert ops.load_ext(), ops.load_error()
    dev = torch.device("cuda", 0)
    model = build_model(a.size, a.ctx, device=dev)
    x = torch.randint(0, 10000, (a.batch, a.ctx), device=dev)

    def step(x):
        with torch.autocast("cuda", dtype=torch.bfloat16):
            return ops.cross_entropy(model(x), x)

    ex = torch._dynamo.explain(step)(x)
    reasons = [f"{getattr(b, 'reason', b)!s:.400} @ {[str(f) for f in getattr(b, 'user_stack', [])][-2:]}"
               for b in ex.break_reasons]
    print(json.dumps({"size": a.size, "graph_count": ex.graph_count, "graph_break_count": ex.graph_break_count,
                      "op_count": ex.op_count, "break_reasons": reasons}, indent=1), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
