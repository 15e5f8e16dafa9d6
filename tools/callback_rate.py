#!/usr/bin/env python3
"""callback_rate.py -- the reference's own call pattern: one frame per call
from host memory, result back in host memory before the call returns
(dips frame_callback, dips/src/lib.rs:233-246; dips_alt send_frame,
dips_alt/src/dips_compute/mod.rs:498-646), 3840x2160 RGBA8.  Output buffers
are preallocated and faulted in; one JSON line per operator."""
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
    from dips_amd.alt import DiPsCompute

    W, H, F = 3840, 2160, int(sys.argv[1]) if len(sys.argv) > 1 else 48
    dev = torch.empty((F, H, W, 4), dtype=torch.uint8, device="cuda")
    op = DiffSeriesOperator(PixelFormat.RGBA8)
    op.synth_device(dev, W, H, 0xD1B5, 0)
    op.close()
    host = dev.cpu().numpy()
    del dev
    out = np.empty((H, W, 4), dtype=np.uint8)
    out.fill(0)

    cs = ComputeState(False, 1, 5.0, DiPsFilter.Unfiltered, ChromaFilter.None_)
    lib, hd = cs._hd._lib, cs._hd
    for t in range(8):  # warm-up: the VecDeque phase and the start texture
        hd.check(lib.dips_frame_callback(hd.ptr, W, H, host[t].ctypes.data, host[t].nbytes, out.ctypes.data, out.nbytes))
    # steady state, the striped call (default) and the plain add_texture +
    # dispatch sequence alternating in rounds (same process, same box)
    times = {"striped": 0.0, "plain": 0.0}
    counts = {"striped": 0, "plain": 0}
    for rnd in range(4):
        for mode in ("striped", "plain"):
            os.environ["DIPS_CALLBACK_STRIPED"] = "1" if mode == "striped" else "0"
            t0 = time.perf_counter()
            for t in range(8, F):
                hd.check(lib.dips_frame_callback(hd.ptr, W, H, host[t].ctypes.data, host[t].nbytes,
                                                 out.ctypes.data, out.nbytes))
            times[mode] += time.perf_counter() - t0
            counts[mode] += F - 8
    os.environ.pop("DIPS_CALLBACK_STRIPED", None)
    cs.close()
    for mode in ("striped", "plain"):
        n, dt = counts[mode], times[mode]
        print(json.dumps({"operator": f"dips frame_callback, one frame per call ({mode})",
                          "frames": n, "frames_per_s": round(n / dt, 1), "ms_per_frame": round(dt / n * 1e3, 3),
                          "pcie_GBps_each_way": round(n * W * H * 4 / dt / 1e9, 1)}), flush=True)

    c = DiPsCompute(2, H, W)
    ha = c._host
    for t in range(4):
        ha.check(ha._lib.dips_alt_send_frame(ha.ptr, host[t].ctypes.data, host[t].nbytes, 0, out.ctypes.data, out.nbytes))
    t0 = time.perf_counter()
    for t in range(4, F):
        ha.check(ha._lib.dips_alt_send_frame(ha.ptr, host[t].ctypes.data, host[t].nbytes, 0, out.ctypes.data, out.nbytes))
    dt = time.perf_counter() - t0
    c.close()
    n = F - 4
    print(json.dumps({"operator": "dips_alt send_frame, one frame per call", "frames": n,
                      "frames_per_s": round(n / dt, 1), "ms_per_frame": round(dt / n * 1e3, 3),
                      "pcie_GBps_each_way": round(n * W * H * 4 / dt / 1e9, 1)}), flush=True)


if __name__ == "__main__":
    main()
