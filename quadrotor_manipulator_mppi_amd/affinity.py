"""Host CPU placement for the launch path.

A control step is two kernel launches whose kernel-argument blocks the host writes into
device memory; on a two-socket host those writes (and the doorbells) cross the socket
link when the launching thread runs on the other socket from the GPU, and the host side
of a step then costs more than the GPU side (measured on the MI355X boxes: 8-11 us of
host enqueue per step from a remote socket against ~6 us from the GPU's own socket, with
a ~9.8 us GPU step).  ``bind_to_gpu_numa`` restricts the calling process to the CPUs the
kernel lists as PCIe-local to the HIP device (``/sys/bus/pci/devices/<bdf>/local_cpulist``;
Linux binds the calling thread, and the threads it creates afterwards inherit the mask),
the usual binding of a GPU-driving process.  It does nothing where the information is
missing (no sysfs entry, a one-socket host) and never widens the current affinity.
"""
from __future__ import annotations

import os
from typing import List, Optional


def _parse_cpulist(s: str) -> List[int]:
    out: List[int] = []
    for part in s.strip().split(","):
        if not part:
            continue
        if "-" in part:
            a, b = part.split("-")
            out.extend(range(int(a), int(b) + 1))
        else:
            out.append(int(part))
    return out


def gpu_pci_bus_id(device: int = 0) -> Optional[str]:
    """The HIP device's PCI address ("0000:75:00.0"), from torch's device properties (the
    process's one HIP runtime: loading libamdhip64 a second time, e.g. through ctypes, can
    hand torch a different runtime than the one it ships with)."""
    try:
        import torch
        if not torch.cuda.is_available() or device >= torch.cuda.device_count():
            return None
        pr = torch.cuda.get_device_properties(device)
        return f"{pr.pci_domain_id:04x}:{pr.pci_bus_id:02x}:{pr.pci_device_id:02x}.0"
    except Exception:   # no GPU, an old torch without the fields
        return None


def gpu_local_cpus(device: int = 0) -> Optional[List[int]]:
    bdf = gpu_pci_bus_id(device)
    if not bdf:
        return None
    try:
        with open(f"/sys/bus/pci/devices/{bdf}/local_cpulist") as f:
            return _parse_cpulist(f.read())
    except OSError:
        return None


def bind_to_gpu_numa(device: int = 0) -> dict:
    """Restrict this process to the GPU's local CPUs (intersected with the current affinity).
    Returns what was done, for the caller's logs."""
    cur = sorted(os.sched_getaffinity(0))
    local = gpu_local_cpus(device)
    info = {"pci_bus_id": gpu_pci_bus_id(device), "cpus_before": len(cur), "bound": False}
    if not local:
        info["reason"] = "no local_cpulist for the device"
        return info
    want = sorted(set(cur) & set(local))
    if not want or len(want) == len(cur):
        info["reason"] = "affinity already local" if want else "no overlap with the current affinity"
        info["cpus_after"] = len(cur)
        return info
    os.sched_setaffinity(0, want)
    info.update(bound=True, cpus_after=len(want), local_cpulist=f"{want[0]}..{want[-1]} ({len(want)} cpus)")
    return info
