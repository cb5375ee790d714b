"""Reference-path module (``cs336_systems/mixed_precision_testing.py``): autocast dtype probe."""

from .bench.precision import ToyModel, autocast_dtypes  # noqa: F401

if __name__ == "__main__":
    import json

    print(json.dumps(autocast_dtypes(), indent=1))
