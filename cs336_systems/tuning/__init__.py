"""Optional per-shape GEMM selections for MI355X (PyTorch TunableOp results: hipBLASLt/rocBLAS
solution per (op, layout, M, N, K, dtype)).

No selection file is committed: on the XL step the TunableOp picks measured within noise of
hipBLASLt's default heuristic (``profiles/r1_overlap_ab.json``), and TunableOp does not cover the
fp32-output weight-gradient GEMMs at all (``CS336_GEMM=lt`` tunes those, ``ops/gemm.py``). So
``bench.py --tunableop auto`` (the default) is OFF unless a file has been produced on the box with
``python bench.py --tunableop tune``, which writes ``tunableop_mi355x.csv`` here; ``--tunableop use``
replays it (TunableOp validates the ROCm/hipBLASLt versions recorded in the file before use)."""

import os

_DIR = os.path.dirname(os.path.abspath(__file__))


def tunableop_file(name: str = "tunableop_mi355x.csv") -> str:
    return os.path.join(_DIR, name)
