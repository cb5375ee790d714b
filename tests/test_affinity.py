"""Per-rank CPU/NUMA affinity helpers (cs336_systems/parallel/affinity.py), on CPU."""

import os

import pytest
import torch

from cs336_systems.parallel import affinity as aff


@pytest.mark.parametrize("text,want", [
    ("0-3", [0, 1, 2, 3]), ("0-3,8,10-11\n", [0, 1, 2, 3, 8, 10, 11]), ("5", [5]), ("", []),
    ("0-7:2", [0, 2, 4, 6]), ("96-101,288-290", list(range(96, 102)) + [288, 289, 290]),
])
def test_parse_cpulist(text, want):
    assert aff.parse_cpulist(text) == want


@pytest.mark.parametrize("cpus,want", [([0, 1, 2, 5], "0-2,5"), ([3], "3"), ([], ""), ([7, 6, 6, 9, 8], "6-9")])
def test_format_cpulist(cpus, want):
    assert aff.format_cpulist(cpus) == want
    assert aff.parse_cpulist(want) == sorted(set(cpus))


def test_pci_address():
    assert aff.pci_address(0, 0x75, 0) == "0000:75:00.0"


def test_gpu_local_cpus_from_sysfs(tmp_path, monkeypatch):
    """A fake sysfs tree: the GPU's PCI address names its local_cpulist."""
    class Prop:
        pci_domain_id, pci_bus_id, pci_device_id = 0, 0x05, 0

    monkeypatch.setattr(torch.cuda, "get_device_properties", lambda i: Prop())
    d = tmp_path / "0000:05:00.0"
    d.mkdir()
    (d / "local_cpulist").write_text("0-3,64-67\n")
    cpus, addr = aff.gpu_local_cpus(0, sysfs=str(tmp_path))
    assert addr == "0000:05:00.0" and cpus == [0, 1, 2, 3, 64, 65, 66, 67]
    assert aff.gpu_local_cpus(0, sysfs=str(tmp_path / "missing"))[0] is None


def test_pin_rank_cpu_device_leaves_mask():
    before = os.sched_getaffinity(0)
    info = aff.pin_rank_to_gpu(torch.device("cpu"))
    assert os.sched_getaffinity(0) == before
    assert info["pinned"] is False and aff.parse_cpulist(info["cpus"]) == sorted(before)
    assert aff.affinity_info()["cpus"] == info["cpus"]
