"""NUMA placement of a rank's host-side work next to its GPU.

The partition logs are pinned host memory that the GPU reads over PCIe (DMA or
zero-copy); on a dual-socket 8-GPU node a log on the far socket pays the inter-socket
link on every byte.  ``bind_to_gpu(dev)`` pins the process's CPUs to the GPU's NUMA node
(from the PCI device's sysfs ``numa_node``), so first-touch and ``hipHostMallocNumaUser``
allocations land on local DRAM.  Best effort: returns the node or None.
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


def gpu_numa_node(device_index: int) -> Optional[int]:
    try:
        import torch
        p = torch.cuda.get_device_properties(device_index)
        bdf = f"{p.pci_domain_id:04x}:{p.pci_bus_id:02x}:{p.pci_device_id:02x}.0"
        with open(f"/sys/bus/pci/devices/{bdf}/numa_node") as f:
            node = int(f.read().strip())
        return node if node >= 0 else None
    except Exception:
        return None


def node_cpus(node: int) -> List[int]:
    try:
        with open(f"/sys/devices/system/node/node{node}/cpulist") as f:
            return _parse_cpulist(f.read())
    except OSError:
        return []


def bind_to_gpu(device_index: int, max_cpus: Optional[int] = None) -> Optional[int]:
    if os.environ.get("CCFD_NO_NUMA_BIND"):
        return None
    node = gpu_numa_node(device_index)
    if node is None:
        return None
    cpus = node_cpus(node)
    try:
        allowed = os.sched_getaffinity(0)
        cpus = [c for c in cpus if c in allowed]
        if max_cpus:
            cpus = cpus[:max_cpus]
        if cpus:
            os.sched_setaffinity(0, cpus)
            return node
    except (AttributeError, OSError):
        pass
    return None
