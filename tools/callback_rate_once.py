#!/usr/bin/env python3
"""callback_rate_once.py -- frames/s of one dips_frame_callback per 4K RGBA8
frame (pageable input and output, DiPsProperties defaults) in this process;
the copy pool size comes from DIPS_COPY_THREADS (read once per process), so
tools/gpu_r03_c6.sh runs it in separate processes per setting."""
from __future__ import annotations

import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    from dips_amd import ChromaFilter, ComputeState, DiffSeriesOperator, DiPsFilter, PixelFormat
    W, H = 3840, 2160
    F = int(sys.argv[1]) if len(sys.argv) > 1 else 64
    dev = torch.empty((F, H, W, 4), dtype=torch.uint8, device="cuda")
    op = DiffSeriesOperator(PixelFormat.RGBA8)
    op.synth_device(dev, W, H, 0xD1B5, 0)
    op.close()
    host = dev.cpu().numpy()
    del dev
    out = np.zeros((H, W, 4), dtype=np.uint8)
    cs = ComputeState(False, 1, 5.0, DiPsFilter.Unfiltered, ChromaFilter.None_)
    lib, hd = cs._hd._lib, cs._hd
    for t in range(8):
        hd.check(lib.dips_frame_callback(hd.ptr, W, H, host[t].ctypes.data, host[t].nbytes, out.ctypes.data, out.nbytes))
    rates = []
    for _ in range(3):
        t0 = time.perf_counter()
        for t in range(8, F):
            hd.check(lib.dips_frame_callback(hd.ptr, W, H, host[t].ctypes.data, host[t].nbytes,
                                             out.ctypes.data, out.nbytes))
        rates.append((F - 8) / (time.perf_counter() - t0))
    cs.close()
    print(json.dumps({"copy_threads": os.environ.get("DIPS_COPY_THREADS", "default"),
                      "frames_per_s": [round(r, 1) for r in rates],
                      "median": round(float(np.median(rates)), 1)}), flush=True)


if __name__ == "__main__":
    main()
