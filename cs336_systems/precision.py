"""Reference-path module (``cs336_systems/precision.py``): fp32/fp16 accumulation demo."""

from .bench.precision import accumulation_demo

if __name__ == "__main__":
    import json

    print(json.dumps(accumulation_demo(), indent=1))
