"""Mixed-precision demonstrations (reference ``precision.py`` and ``mixed_precision_testing.py``;
handout §1.1.5).

* :func:`accumulation_demo` — summing 0.01 one thousand times in fp32, fp16, and fp16 with an fp32
  accumulator, showing why reductions keep fp32 accumulators (what every HIP kernel here does).
* :func:`autocast_dtypes` — which dtype each piece of a ToyModel (fc1 → ReLU → LayerNorm → fc2)
  produces under ``torch.autocast`` (bf16 on MI355X): parameters stay fp32, linear outputs are
  bf16, LayerNorm runs in fp32, logits bf16, loss fp32, gradients fp32.

    python -m cs336_systems.bench.precision
"""

from __future__ import annotations

import json

import torch
import torch.nn as nn


def accumulation_demo() -> dict:
    out = {}
    s = torch.tensor(0, dtype=torch.float32)
    for _ in range(1000):
        s += torch.tensor(0.01, dtype=torch.float32)
    out["fp32 += fp32"] = float(s)
    s = torch.tensor(0, dtype=torch.float16)
    for _ in range(1000):
        s += torch.tensor(0.01, dtype=torch.float16)
    out["fp16 += fp16"] = float(s)
    s = torch.tensor(0, dtype=torch.float32)
    for _ in range(1000):
        s += torch.tensor(0.01, dtype=torch.float16)
    out["fp32 += fp16"] = float(s)
    s = torch.tensor(0, dtype=torch.float32)
    for _ in range(1000):
        s += torch.tensor(0.01, dtype=torch.float16).type(torch.float32)
    out["fp32 += fp16->fp32"] = float(s)
    return out


class ToyModel(nn.Module):
    def __init__(self, in_features: int = 16, out_features: int = 8):
        super().__init__()
        self.fc1 = nn.Linear(in_features, 10, bias=False)
        self.ln = nn.LayerNorm(10)
        self.fc2 = nn.Linear(10, out_features, bias=False)
        self.relu = nn.ReLU()
        self.trace: dict[str, str] = {}

    def forward(self, x):
        h = self.fc1(x)
        self.trace["fc1 output"] = str(h.dtype)
        h = self.relu(h)
        h = self.ln(h)
        self.trace["layernorm output"] = str(h.dtype)
        y = self.fc2(h)
        self.trace["logits"] = str(y.dtype)
        return y


def autocast_dtypes(device=None, dtype=torch.bfloat16) -> dict:
    dev = device or ("cuda" if torch.cuda.is_available() else "cpu")
    m = ToyModel().to(dev)
    x = torch.randn(4, 16, device=dev)
    with torch.autocast(torch.device(dev).type, dtype=dtype):
        y = m(x)
        loss = torch.nn.functional.cross_entropy(y, torch.zeros(4, dtype=torch.long, device=dev))
    loss.backward()
    out = dict(m.trace)
    out["parameters"] = str(m.fc1.weight.dtype)
    out["loss"] = str(loss.dtype)
    out["gradients"] = str(m.fc1.weight.grad.dtype)
    return out


def main():
    print(json.dumps({"accumulation": accumulation_demo(), "autocast": autocast_dtypes()}, indent=1))


if __name__ == "__main__":
    main()
