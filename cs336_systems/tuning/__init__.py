"""Committed per-shape GEMM selections for MI355X (PyTorch TunableOp results: hipBLASLt/rocBLAS
solution per (op, layout, M, N, K, dtype)). Produced with ``python bench.py --tunableop tune`` on
an MI355X with this image's ROCm/hipBLASLt, replayed with ``--tunableop use`` (the default when the
file exists). TunableOp validates the ROCm/hipBLASLt versions recorded in the file before use."""

import os

_DIR = os.path.dirname(os.path.abspath(__file__))


def tunableop_file(name: str = "tunableop_mi355x.csv") -> str:
    return os.path.join(_DIR, name)
