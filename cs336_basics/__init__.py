"""cs336_basics API (the reference's bundled staff package plus the student modules its systems
code imports: ``transformer``, ``optimizers``, ``training``). Implementation
lives in ``cs336_systems.models`` / ``cs336_systems.ops``; these modules keep the import paths."""

import importlib.metadata as _md

try:
    __version__ = _md.version("cs336_basics")
except _md.PackageNotFoundError:  # in-tree use
    __version__ = "1.0.3"

from .model import BasicsTransformerLM  # noqa: E402,F401
