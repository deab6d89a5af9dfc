"""Host side of the launch path (tools/): the process's CPU affinity, the GPU's PCIe-local
CPUs / NUMA node, and run_steps' host enqueue rate with the process bound to local vs
non-local CPUs.   python tools/host_affinity_probe.py"""
import glob
import json
import os
import subprocess
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch
    info = {"affinity": sorted(os.sched_getaffinity(0)), "cpu_count": os.cpu_count()}
    props = torch.cuda.get_device_properties(0)
    bdf = None
    for attr in ("pci_bus_id",):
        bdf = getattr(props, attr, None)
    info["gpu_name"] = props.name
    # the GPU's PCI function: the render node behind HIP device 0 (first amdgpu card with a numa_node)
    cards = []
    for d in sorted(glob.glob("/sys/class/drm/card*/device")):
        try:
            vendor = open(os.path.join(d, "vendor")).read().strip()
        except OSError:
            continue
        if vendor != "0x1002":
            continue
        def rd(n):
            try:
                return open(os.path.join(d, n)).read().strip()
            except OSError:
                return None
        cards.append({"dev": os.path.realpath(d), "numa_node": rd("numa_node"), "local_cpulist": rd("local_cpulist")})
    info["amd_cards"] = cards
    print(json.dumps(info), flush=True)


if __name__ == "__main__":
    main()
