#!/usr/bin/env python3
"""stripe_trace.py -- host timeline of the striped per-frame call
(dips_frame_callback, host_stream.h run_striped_frame) with
DIPS_STRIPE_TRACE=1: per stripe [staged, DMA enqueued, readback landed,
copied out] in us from the call's entry, for the DMA form (4 MiB) and the zero-copy form (2 and 4 MiB stripes),
4K RGBA8; DIPS_COPY_THREADS sets the copy pool size."""
from __future__ import annotations

import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
os.environ["DIPS_STRIPE_TRACE"] = "1"


def main():
    import torch
    from dips_amd import ChromaFilter, ComputeState, DiffSeriesOperator, DiPsFilter, PixelFormat

    W, H, F = 3840, 2160, 24
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
    for direct, piece in (("0", 4 << 20), ("1", 4 << 20)):
        os.environ["DIPS_CALLBACK_DIRECT"] = direct
        os.environ["DIPS_PIECE_BYTES"] = str(piece)
        print(f"== direct {direct} piece {piece >> 20} MiB", file=sys.stderr, flush=True)
        t0 = time.perf_counter()
        for t in range(8, F):
            hd.check(lib.dips_frame_callback(hd.ptr, W, H, host[t].ctypes.data, host[t].nbytes,
                                             out.ctypes.data, out.nbytes))
        dt = time.perf_counter() - t0
        print(f"== direct {direct} piece {piece >> 20} MiB: {(F - 8) / dt:.1f} frames/s", file=sys.stderr, flush=True)
    cs.close()


if __name__ == "__main__":
    main()
