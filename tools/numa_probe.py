#!/usr/bin/env python3
"""numa_probe.py -- where the per-frame call's memory lives on the GPU box:
the GPU's NUMA node, the node layout and this process's CPU affinity, and
the per-node page counts (/proc/self/numa_maps) of the pinned staging
buffers libdips_hip.so allocates for a 4K frame_callback, of a pageable
numpy frame, and of a torch pinned tensor.  Read-only queries; one JSON
line."""
from __future__ import annotations

import glob
import json
import os
import re
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def read(p):
    try:
        with open(p) as f:
            return f.read().strip()
    except OSError:
        return None


def numa_maps(min_bytes=8 << 20):
    out = []
    txt = read("/proc/self/numa_maps") or ""
    for line in txt.splitlines():
        nodes = {k: int(v) for k, v in re.findall(r"\bN(\d+)=(\d+)", line)}
        pages = sum(nodes.values())
        kps = re.search(r"kernelpagesize_kB=(\d+)", line)
        kb = int(kps.group(1)) if kps else 4
        if pages * kb * 1024 >= min_bytes:
            out.append({"addr": line.split()[0], "policy": line.split()[1], "MB": round(pages * kb / 1024, 1),
                        "pages_per_node": nodes, "page_kB": kb, "anon": "anon=" in line,
                        "file": (re.search(r"file=(\S+)", line) or [None, None])[1]})
    return out


def main():
    import torch
    from dips_amd import ChromaFilter, ComputeState, DiPsFilter
    props = torch.cuda.get_device_properties(0)
    bus = f"{props.pci_domain_id:04x}:{props.pci_bus_id:02x}:{props.pci_device_id:02x}.0"
    nodes = {os.path.basename(n): read(n + "/cpulist") for n in sorted(glob.glob("/sys/devices/system/node/node*"))}
    rec = {"gpu_pci": bus, "gpu_numa_node": read(f"/sys/bus/pci/devices/{bus}/numa_node"), "nodes": nodes,
           "affinity_n": len(os.sched_getaffinity(0)), "cpu_now": os.sched_getaffinity(0) and None,
           "cgroup_cpu_max": read("/sys/fs/cgroup/cpu.max"), "cpuset_effective": read("/sys/fs/cgroup/cpuset.cpus.effective"),
           "mems_effective": read("/sys/fs/cgroup/cpuset.mems.effective")}
    try:
        with open("/proc/self/stat") as f:
            rec["cpu_now"] = int(f.read().split()[38])
    except (OSError, ValueError, IndexError):
        pass
    before = {m["addr"] for m in numa_maps()}
    W, H = 3840, 2160
    frame = np.random.default_rng(0).integers(0, 256, (H, W, 4), dtype=np.uint8)
    out = np.empty_like(frame)
    cs = ComputeState(False, 1, 5.0, DiPsFilter.Unfiltered, ChromaFilter.None_)
    from dips_amd import frame_callback
    for _ in range(8):
        frame_callback(W, H, frame, cs)
    pinned = torch.empty(64 << 20, dtype=torch.uint8, pin_memory=True)
    pinned.fill_(1)
    rec["mappings_new"] = [m for m in numa_maps() if m["addr"] not in before]
    rec["numpy_frame_addr"] = hex(frame.ctypes.data)
    rec["torch_pinned_addr"] = hex(pinned.data_ptr())
    cs.close()
    print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
