"""Student ``cs336_basics.optimizers`` API (``benchmark.py:4``): AdamW + cosine schedule."""

from .optimizer import AdamW, ReferenceAdamW, get_cosine_lr  # noqa: F401

get_lr_cosine_schedule = get_cosine_lr
