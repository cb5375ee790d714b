import os

import numpy as np
import pytest

os.environ.setdefault("MASTER_ADDR", "127.0.0.1")

SNAPSHOT_DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)), "_snapshots")


def pytest_addoption(parser):
    parser.addoption("--snapshot-exact", action="store_true", help="snapshot comparisons require bit equality")
    parser.addoption("--update-snapshots", action="store_true", help="(re)write snapshot files instead of comparing")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP) GPU and the built extension")


def pytest_collection_modifyitems(config, items):
    import torch

    if torch.cuda.is_available():
        return
    skip = pytest.mark.skip(reason="no GPU in this environment")
    for item in items:
        if "gpu" in item.keywords:
            item.add_marker(skip)


class NumpySnapshot:
    """Compare named arrays with ``tests/_snapshots/<name>.npz`` (the reference's
    ``numpy_snapshot`` fixture, ``tests/conftest.py:25-190`` there, re-designed: one ``.npz`` per
    snapshot, loaded with ``allow_pickle=False``). ``--snapshot-exact`` demands bit equality;
    ``--update-snapshots`` writes the file instead of comparing."""

    def __init__(self, exact: bool, update: bool):
        self.exact, self.update = exact, update

    def assert_match(self, arrays: dict, name: str, rtol: float = 1e-4, atol: float = 1e-6) -> None:
        path = os.path.join(SNAPSHOT_DIR, name + ".npz")
        arrays = {k: np.asarray(v.detach().cpu().numpy() if hasattr(v, "detach") else v) for k, v in arrays.items()}
        if self.update or not os.path.exists(path):
            if not self.update:
                pytest.fail(f"snapshot {path} missing (run with --update-snapshots to create it)")
            os.makedirs(SNAPSHOT_DIR, exist_ok=True)
            np.savez(path, **arrays)
            return
        with np.load(path, allow_pickle=False) as ref:
            assert set(ref.files) == set(arrays), (sorted(ref.files), sorted(arrays))
            for k, v in arrays.items():
                if self.exact:
                    np.testing.assert_array_equal(v, ref[k], err_msg=k)
                else:
                    np.testing.assert_allclose(v, ref[k], rtol=rtol, atol=atol, err_msg=k)


@pytest.fixture
def numpy_snapshot(request):
    return NumpySnapshot(request.config.getoption("--snapshot-exact"), request.config.getoption("--update-snapshots"))


@pytest.fixture
def snapshot(numpy_snapshot):
    """Tensor alias of :func:`numpy_snapshot` (torch tensors are converted on the way in)."""
    return numpy_snapshot
