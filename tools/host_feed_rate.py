#!/usr/bin/env python3
"""host_feed_rate.py -- PCIe-inclusive rate of the visual operators from
host (pageable) frames: dips_frame_callback_batch (dips ComputeState) and
dips_alt_run (dips_alt loop), 3840x2160 RGBA8, both directions over PCIe
(frames up, RGBA8 outputs down), pipelined in ~256 MiB chunks.  Reported
beside, never as, the HBM-resident kernel rates.  One JSON line per operator.
"""
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
    from dips_amd.alt import DiPsRunner

    W, H, F = 3840, 2160, int(sys.argv[1]) if len(sys.argv) > 1 else 160
    dev = torch.empty((F, H, W, 4), dtype=torch.uint8, device="cuda")
    op = DiffSeriesOperator(PixelFormat.RGBA8)
    op.synth_device(dev, W, H, 0xD1B5, 0)
    op.close()
    host = dev.cpu().numpy()
    del dev
    fb = W * H * 4
    # one output buffer, faulted in before timing: releasing a multi-GB numpy
    # result (munmap of its pages) costs ~40 ms/GB on the box and is not
    # part of the operator
    out = np.empty_like(host)
    out.fill(0)

    def cb(o, x):
        o._hd.check(o._hd._lib.dips_frame_callback_batch(o._hd.ptr, W, H, x.ctypes.data, x.shape[0], out.ctypes.data))

    def run(o, x):
        h = o.compute._host
        h.check(h._lib.dips_alt_run(h.ptr, x.ctypes.data, x.shape[0], None, 0, out.ctypes.data))

    for name, make, call in [
        ("dips ComputeState frame_callback_batch",
         lambda: ComputeState(False, 1, 5.0, DiPsFilter.Unfiltered, ChromaFilter.None_), cb),
        ("dips_alt run loop", lambda: DiPsRunner(H, W), run),
    ]:
        obj = make()
        call(obj, host[:16])  # warm-up (allocations, first frames of the stream)
        t = time.perf_counter()
        call(obj, host)
        dt = time.perf_counter() - t
        obj.close()
        print(json.dumps({"operator": name, "frames": F, "frames_per_s": round(F / dt, 1),
                          "host_to_device_GBps": round(F * fb / dt / 1e9, 1),
                          "device_to_host_GBps": round(F * fb / dt / 1e9, 1),
                          "output_shape": list(out.shape)}), flush=True)


if __name__ == "__main__":
    main()
