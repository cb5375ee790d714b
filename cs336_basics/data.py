"""Batch sampling from a token array (reference ``data.py:10-30``)."""

from cs336_systems.data import get_batch  # noqa: F401
