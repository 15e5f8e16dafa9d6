#!/usr/bin/env python3
"""pin_huge_ab.py -- the per-frame call (dips_frame_callback, 4K RGBA8, one
frame per call from pageable memory) with its pinned staging / output
buffers from hipHostMalloc (DIPS_PIN_HUGE=0) against 2 MiB transparent huge
pages registered with hipHostRegister (=1): one handle each (the buffers are
allocated at the handle's first frames), alternated over rounds in one
process; outputs compared between the two."""
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
    F = int(sys.argv[1]) if len(sys.argv) > 1 else 40
    rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 4
    dev = torch.empty((F, H, W, 4), dtype=torch.uint8, device="cuda")
    op = DiffSeriesOperator(PixelFormat.RGBA8)
    op.synth_device(dev, W, H, 0xD1B5, 0)
    op.close()
    host = dev.cpu().numpy()
    del dev
    outs = {}
    handles = {}
    for name, env in (("hipHostMalloc", "0"), ("huge pages", "1")):
        os.environ["DIPS_PIN_HUGE"] = env
        cs = ComputeState(False, 1, 5.0, DiPsFilter.Unfiltered, ChromaFilter.None_)
        out = np.zeros((H, W, 4), dtype=np.uint8)
        lib, hd = cs._hd._lib, cs._hd
        for t in range(8):  # allocates the pinned buffers under this setting
            hd.check(lib.dips_frame_callback(hd.ptr, W, H, host[t].ctypes.data, host[t].nbytes, out.ctypes.data,
                                             out.nbytes))
        handles[name] = (cs, out)
    os.environ.pop("DIPS_PIN_HUGE", None)
    res = {}
    for rnd in range(rounds):
        names = list(handles) if rnd % 2 == 0 else list(handles)[::-1]
        for name in names:
            cs, out = handles[name]
            lib, hd = cs._hd._lib, cs._hd
            seq = list(range(F - 3, F)) + list(range(8, F))
            t0 = time.perf_counter()
            got = []
            for pos, t in enumerate(seq):
                hd.check(lib.dips_frame_callback(hd.ptr, W, H, host[t].ctypes.data, host[t].nbytes,
                                                 out.ctypes.data, out.nbytes))
                if pos == len(seq) - 1:
                    got.append(out.copy())
            dt = time.perf_counter() - t0
            outs.setdefault(name, got[-1])
            res.setdefault(name, []).append(len(seq) / dt)
            print(json.dumps({"variant": name, "round": rnd, "frames_per_s": round(len(seq) / dt, 1)}), flush=True)
    same = bool(np.array_equal(*outs.values()))
    for k, v in res.items():
        print(json.dumps({"variant": k, "summary": True, "median_frames_per_s": round(float(np.median(v)), 1),
                          "outputs_equal_other": same}), flush=True)
    for cs, _ in handles.values():
        cs.close()


if __name__ == "__main__":
    main()
