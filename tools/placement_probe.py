#!/usr/bin/env python3
"""placement_probe.py -- where a 124 GB frame buffer lands in HBM, and what
that costs the headline kernel.

Round 3 found two 124 GB buffers of one process 2.5-3 points apart whatever
their memory type (HISTORY.md, "Open items after round 3"); round 5 saw
consecutive bench processes alternate between ~72.5 % and ~74.7 %
(`profiles/r05/ab_u5/`).  This allocates two such buffers in one process
(A, then B; 249 GB of the 288 GB), fills both with the bench's frames, and
for each reports: the series kernel's rate (the bench's 4K per-frame batch,
a few launches), the compute-free read of the whole buffer, and the
compute-free read of each of 16 equal slices -- so a slow region of the
address space, if there is one, shows as slow slices.  Then B is freed, a
third buffer C takes its place, and C is measured too.

Run on the GPU box: python tools/placement_probe.py [--launches 3] [--vmm | --pair vd]
"""
from __future__ import annotations

import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

W, H, C, F = 3840, 2160, 3, 5000
SEED = 0xD1B5


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--launches", type=int, default=3)
    ap.add_argument("--slices", type=int, default=16)
    ap.add_argument("--vmm", action="store_true", help="buffers through the HIP virtual-memory API instead")
    ap.add_argument("--pair", default="", help="e.g. 'vd' / 'dv': a 1 GiB-aligned virtual-memory buffer (v) and a "
                    "torch one (d), allocated in this order, then measured alternately, twice each")
    args = ap.parse_args()
    import numpy as np
    import torch
    from dips_amd import DiffSeriesOperator, Mode, PixelFormat

    dev = torch.device("cuda", 0)
    op = DiffSeriesOperator(PixelFormat.RGB8, Mode.PerFrame, 8 / 255, time_kernel=True)
    fb = W * H * C

    def measure(name, buf):
        frames = buf.view(F, H, W, C)
        op.synth_device(frames, W, H, SEED, 0)
        series = torch.zeros((F, 4), dtype=torch.int64, device=dev)
        op.run_device(frames, series)
        torch.cuda.synchronize()
        op.kernel_time(reset=True)
        for _ in range(args.launches):
            op.run_device(frames, series)
        torch.cuda.synchronize()
        ms, n = op.kernel_time()
        ms /= max(n, 1)
        whole = float(np.median([op.read_ceiling_ms(buf) for _ in range(3)]))
        step = buf.numel() // args.slices // 4096 * 4096
        sl = []
        for k in range(args.slices):
            part = buf[k * step:(k + 1) * step]
            t = float(np.median([op.read_ceiling_ms(part) for _ in range(3)]))
            sl.append(round(step / (t / 1e3) / 1e9, 1))
        rec = {"buffer": name, "device_address_GiB": round(buf.data_ptr() / 2 ** 30, 2),
               "series_frac_of_8TBps": round(F * fb / (ms / 1e3) / 8e12, 4), "series_ms": round(ms, 4),
               "read_GBps": round(buf.numel() / (whole / 1e3) / 1e9, 1), "slice_read_GBps": sl,
               "slice_GB": round(step / 1e9, 2)}
        print(json.dumps(rec), flush=True)

    if not args.vmm and not args.pair:
        a = torch.empty(F * fb, dtype=torch.uint8, device=dev)
        b = torch.empty(F * fb, dtype=torch.uint8, device=dev)
        measure("A", a)
        measure("B", b)
        measure("A again", a)
        del b
        torch.cuda.empty_cache()
        c = torch.empty(F * fb, dtype=torch.uint8, device=dev)
        measure("C (after freeing B)", c)
        op.close()
        return
    # the same frames in buffers made through the virtual-memory API
    # (tools/vmm_probe.hip): virtual alignment x physical chunk size
    import ctypes
    vmm = ctypes.CDLL(os.path.join(ROOT, "tools", "libvmm_probe.so"))
    vmm.vmm_granularity.restype = ctypes.c_size_t
    vmm.vmm_granularity.argtypes = [ctypes.c_int]
    vmm.vmm_alloc.argtypes = [ctypes.c_int, ctypes.c_size_t, ctypes.c_size_t, ctypes.c_size_t,
                              ctypes.POINTER(ctypes.c_void_p)]
    vmm.vmm_free.argtypes = [ctypes.c_int]
    gran = vmm.vmm_granularity(0)
    print(json.dumps({"granularity": gran}), flush=True)
    GiB, MiB = 1 << 30, 1 << 20
    size = -(-F * fb // GiB) * GiB

    class _Dev:
        def __init__(self, ptr, n):
            self.__cuda_array_interface__ = {"shape": (n,), "typestr": "|u1", "data": (ptr, False), "version": 3}

    if args.pair:
        bufs = []
        for kind in args.pair:
            if kind == "d":
                bufs.append(("torch default", torch.empty(F * fb, dtype=torch.uint8, device=dev)))
                continue
            ptr = ctypes.c_void_p()
            bid = vmm.vmm_alloc(0, size, GiB, size, ctypes.byref(ptr))
            if bid < 0:
                raise SystemExit(f"vmm_alloc failed: {bid}")
            bufs.append(("vmm: 1 GiB-aligned, one physical allocation",
                         torch.as_tensor(_Dev(ptr.value, size), device=dev)[: F * fb]))
        for rep in range(2):
            for idx, (name, buf) in enumerate(bufs):
                measure(f"{name} (allocated #{idx}, pass {rep})", buf)
        del bufs
        torch.cuda.synchronize()
        op.close()
        return
    for name, align, chunk in (("vmm: 1 GiB-aligned, one physical allocation", GiB, size),
                               ("vmm: 2 MiB-aligned, one physical allocation", 2 * MiB, size),
                               ("vmm: 1 GiB-aligned, 1 GiB physical chunks", GiB, GiB),
                               ("vmm: 1 GiB-aligned, 64 MiB physical chunks", GiB, 64 * MiB),
                               ("torch default (for comparison)", 0, 0)):
        if chunk == 0:
            buf = torch.empty(F * fb, dtype=torch.uint8, device=dev)
            measure(name, buf)
            del buf
            torch.cuda.empty_cache()
            continue
        ptr = ctypes.c_void_p()
        bid = vmm.vmm_alloc(0, size, align, chunk, ctypes.byref(ptr))
        if bid < 0:
            print(json.dumps({"buffer": name, "failed": bid}), flush=True)
            continue
        buf = torch.as_tensor(_Dev(ptr.value, size), device=dev)[: F * fb]
        measure(name, buf)
        del buf
        torch.cuda.synchronize()
        vmm.vmm_free(bid)
    op.close()


if __name__ == "__main__":
    main()
