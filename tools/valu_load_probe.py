#!/usr/bin/env python3
"""valu_load_probe.py -- HBM rate and package power of a full-rate stream as
a function of the VALU work per byte (tools/valu_load_probe.hip).

For K in (0, 1, 2, 4, ..., 24) v_fma_f32 per loaded dword (with the 3 ops
that make and fold the value, 0.75 (K + 3) VALU ops per RGB8 pixel), `--launches` back-to-back launches over a resident 24.9 GB buffer
(1000 4K RGB8 frames' worth), timed with hipEvents on the launch stream and
bracketed by readings of the energy counter, PPT residency and gfx clock
(tools/power_probe.py Sampler, as bench.py's power legs).  One JSON line per
K: GB/s, fraction of 8 TB/s, ops per pixel, average W, PPT residency, clock.

The question it answers: at how many VALU ops per byte does the stream start
to lose bandwidth to the power limit, and is the series kernel's ~12.75-13.65 ops
per pixel past that point?

Build (here):  hipcc --offload-arch=gfx950 -O3 -shared -fPIC -cuid=valu_load_probe \\
                 -o tools/libvalu_load_probe.so tools/valu_load_probe.hip
Run (GPU box): python tools/valu_load_probe.py [--launches 60]
"""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))

KS = (0, 1, 2, 4, 6, 8, 10, 12, 16, 20, 24)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--launches", type=int, default=60)
    ap.add_argument("--gb", type=float, default=24.8832, help="buffer size (GB)")
    args = ap.parse_args()
    import torch
    from power_probe import Sampler

    lib = ctypes.CDLL(os.path.join(ROOT, "tools", "libvalu_load_probe.so"))
    lib.valu_load_launch.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_int, ctypes.c_void_p,
                                     ctypes.c_void_p]
    lib.valu_load_launch.restype = ctypes.c_int
    dev = torch.device("cuda", 0)
    nbytes = int(args.gb * 1e9) // 16 * 16
    buf = torch.randint(0, 2 ** 31 - 1, (nbytes // 4,), dtype=torch.int32, device=dev)
    out = torch.empty(1024 * 256, dtype=torch.float32, device=dev)
    stream = torch.cuda.current_stream(dev)
    smp = Sampler(pci_bus=torch.cuda.get_device_properties(0).pci_bus_id)
    if len(smp.handles) != 1:
        smp = None

    def run(k, n):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        for _ in range(n):
            if lib.valu_load_launch(buf.data_ptr(), nbytes, k, out.data_ptr(), stream.cuda_stream) != 0:
                raise RuntimeError(f"launch failed for K = {k}")
        e1.record(stream)
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) / n

    for k in KS:
        run(k, 2)  # warm
        rec = {"K_fma_per_dword": k, "valu_ops_per_rgb8_px": round(0.75 * (k + 3), 2), "launches": args.launches,
               "bytes_per_launch": nbytes}
        if smp is not None:
            smp.sample()
            ta = smp.rows[-1][0]
        ms = run(k, args.launches)
        if smp is not None:
            smp.sample()
            tb = smp.rows[-1][0]
            g = smp.window(ta, tb)[0] or {}
            rec["power"] = {"avg_W": g.get("avg_power_W_energy"), "ppt_throttle_residency": g.get("ppt_residency_frac"),
                            "gfxclk_MHz_before_after": [r[4] for r in smp.rows if ta <= r[0] <= tb],
                            "seconds": round(tb - ta, 3)}
        rec["ms_per_launch"] = round(ms, 4)
        rec["GBps"] = round(nbytes / (ms / 1e3) / 1e9, 1)
        rec["frac_of_8TBps"] = round(nbytes / (ms / 1e3) / 8e12, 4)
        print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
