"""Reference-path module (``cs336_systems/transformer_annotated.py``): the Transformer LM with roctx
ranges on every block / attention / projection / FFN (visible in ``rocprofv3 --marker-trace``).

The model itself carries the ranges (``cs336_systems/models/transformer.py`` ``annotate(...)``);
importing this module switches them on (the reference's monkeypatch never took effect)."""

from .models.transformer import *  # noqa: F401,F403
from .models.transformer import BasicsTransformerLM  # noqa: F401
from .utils.profiling import enable_annotations

enable_annotations(True)
