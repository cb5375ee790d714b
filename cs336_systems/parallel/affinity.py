"""Per-rank CPU / NUMA affinity (SURVEY §7.5 scaling hygiene; the reference has none).

An 8-GPU MI355X node has several NUMA domains, and each GPU hangs off one of them. A rank whose
host threads (autograd engine, DDP hooks, RCCL proxy threads, pinned-memory copies) run on a remote
domain pays cross-socket memory traffic and scheduling jitter on every launch. So each rank pins its
process to the CPUs local to its GPU before any heavy host work: the GPU's PCI address (from the
device properties) names ``/sys/bus/pci/devices/<addr>/local_cpulist``, intersected with the CPUs this
process may use at all (a container's cpuset). ``CS336_NUMA_PIN=0`` disables it.
"""

from __future__ import annotations

import os

_STATE: dict = {}


def parse_cpulist(text: str) -> list[int]:
    """Linux cpulist syntax (``"0-3,8,10-11"``, stride form ``"0-15:2"``) -> sorted CPU ids."""
    cpus: set[int] = set()
    for part in text.strip().split(","):
        part = part.strip()
        if not part:
            continue
        stride = 1
        if ":" in part:
            part, s = part.split(":", 1)
            stride = int(s)
        if "-" in part:
            lo, hi = part.split("-", 1)
            cpus.update(range(int(lo), int(hi) + 1, stride))
        else:
            cpus.add(int(part))
    return sorted(cpus)


def format_cpulist(cpus) -> str:
    """Sorted CPU ids -> compact cpulist (``[0, 1, 2, 5]`` -> ``"0-2,5"``)."""
    cpus = sorted(set(cpus))
    out, i = [], 0
    while i < len(cpus):
        j = i
        while j + 1 < len(cpus) and cpus[j + 1] == cpus[j] + 1:
            j += 1
        out.append(str(cpus[i]) if i == j else f"{cpus[i]}-{cpus[j]}")
        i = j + 1
    return ",".join(out)


def pci_address(domain: int, bus: int, device: int, function: int = 0) -> str:
    return f"{domain:04x}:{bus:02x}:{device:02x}.{function:x}"


def gpu_local_cpus(device_index: int, sysfs: str = "/sys/bus/pci/devices") -> tuple[list[int] | None, str]:
    """CPUs local to GPU ``device_index`` and the PCI address they came from (None if unknown)."""
    import torch

    try:
        prop = torch.cuda.get_device_properties(device_index)
        addr = pci_address(int(getattr(prop, "pci_domain_id", 0)), int(prop.pci_bus_id), int(prop.pci_device_id))
    except Exception:  # noqa: BLE001 - no GPU / no PCI info: nothing to pin to
        return None, ""
    path = os.path.join(sysfs, addr, "local_cpulist")
    try:
        with open(path) as f:
            return parse_cpulist(f.read()), addr
    except OSError:
        return None, addr


def _pin_all_threads(cpus: list[int]) -> tuple[int, int]:
    """Set ``cpus`` as the affinity of every thread in /proc/self/task; (threads set, threads seen)."""
    try:
        tids = [int(t) for t in os.listdir("/proc/self/task")]
    except OSError:
        return 0, 0
    ok = 0
    for tid in tids:
        try:
            os.sched_setaffinity(tid, cpus)
            ok += 1
        except OSError:  # the thread exited meanwhile, or is not ours to move
            pass
    return ok, len(tids)


def pin_rank_to_gpu(device) -> dict:
    """Pin this process (every thread of it) to the CPUs local to ``device`` (a CUDA/HIP device); returns what happened
    (also kept for :func:`affinity_info`). CPU devices and unknown topologies leave the mask as is."""
    info: dict = {"pinned": False}
    try:
        allowed = sorted(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        allowed = []
    if getattr(device, "type", "cpu") == "cuda" and os.environ.get("CS336_NUMA_PIN", "1") != "0" and allowed:
        idx = device.index if device.index is not None else 0
        local, addr = gpu_local_cpus(idx)
        info["gpu_pci"] = addr
        if local:
            want = sorted(set(local) & set(allowed))
            info["gpu_local_cpus"] = format_cpulist(local)
            if want and want != allowed:
                try:
                    os.sched_setaffinity(0, want)
                    info["pinned"] = True
                except OSError as e:
                    info["error"] = str(e)
                # sched_setaffinity(0) pins only the calling thread: the HIP runtime's threads (and an
                # OpenMP pool) started before this call keep the full mask, so apply it to every
                # thread of the process and report how many took it
                n_ok, n_all = _pin_all_threads(want)
                info["threads_pinned"] = f"{n_ok}/{n_all}"
            elif want:
                info["pinned"] = True  # already exactly the local set
    try:
        info["cpus"] = format_cpulist(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        info["cpus"] = ""
    _STATE.clear()
    _STATE.update(info)
    return info


def affinity_info() -> dict:
    """This process's affinity as set up by :func:`pin_rank_to_gpu` (or the current mask)."""
    if _STATE:
        return dict(_STATE)
    try:
        return {"pinned": False, "cpus": format_cpulist(os.sched_getaffinity(0))}
    except (AttributeError, OSError):
        return {"pinned": False, "cpus": ""}
