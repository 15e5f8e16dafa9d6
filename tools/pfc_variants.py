#!/usr/bin/env python3
"""pfc_variants.py -- why the bench's per_frame_call leg runs slower than the
A/B tools: the same 4K RGBA8 frame_callback loop (208 frames) with an output
compare between calls (the bench leg's old form), without it, and with every
output written to its own pre-faulted buffer and compared after the loop."""
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
    W, H, n = 3840, 2160, 208
    gen = DiffSeriesOperator(PixelFormat.RGBA8)
    dev = torch.empty((n, H, W, 4), dtype=torch.uint8, device="cuda")
    gen.synth_device(dev, W, H, 0xD1B5 ^ 0x4A, 0)
    gen.close()
    host = dev.cpu().numpy()
    b = ComputeState(False, 1, 5.0, DiPsFilter.Unfiltered, ChromaFilter.None_)
    od = torch.empty_like(dev)
    b.frame_callback_batch_device(dev, od)
    torch.cuda.synchronize()
    want = od.cpu().numpy()
    b.close()
    del dev, od
    torch.cuda.empty_cache()
    outs = np.empty_like(host)
    outs.fill(0)
    for variant in ("compare between calls", "no compare", "own buffers, compare after", "compare between calls",
                    "no compare", "own buffers, compare after"):
        cs = ComputeState(False, 1, 5.0, DiPsFilter.Unfiltered, ChromaFilter.None_)
        lib, hd = cs._hd._lib, cs._hd
        out = np.zeros((H, W, 4), dtype=np.uint8)
        times, ok = [], True
        for t in range(n):
            dst = outs[t] if variant.startswith("own") else out
            t0 = time.perf_counter()
            hd.check(lib.dips_frame_callback(hd.ptr, W, H, host[t].ctypes.data, host[t].nbytes,
                                             dst.ctypes.data, dst.nbytes))
            if t >= 8:
                times.append(time.perf_counter() - t0)
            if variant.startswith("compare"):
                ok = ok and bool(np.array_equal(out, want[t]))
        if variant.startswith("own"):
            ok = bool(np.array_equal(outs, want))
        cs.close()
        print(json.dumps({"variant": variant, "frames_per_s": round(len(times) / sum(times), 1),
                          "median_ms": round(float(np.median(times)) * 1e3, 4), "equal": ok}), flush=True)


if __name__ == "__main__":
    main()
