#!/usr/bin/env python3
"""window_callback_rate.py -- dips frame_callback, one 4K RGBA8 frame per
call (the reference's own pattern), for spatial windows 1/3/5/11: the
deferred add_texture (staged frame, speculative dispatch; default) against
DMA upload + DMA readback (DIPS_DEFER_UPLOAD=0, and DIPS_CALLBACK_STRIPED=0
so that W = 1 takes the same add_texture + dispatch route), alternated in one
process.  Outputs of the two forms are compared on the last frame."""
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

    W, H, F = 3840, 2160, 28
    dev = torch.empty((F, H, W, 4), dtype=torch.uint8, device="cuda")
    op = DiffSeriesOperator(PixelFormat.RGBA8)
    op.synth_device(dev, W, H, 0xD1B5, 0)
    op.close()
    host = dev.cpu().numpy()
    del dev
    out = np.zeros((H, W, 4), dtype=np.uint8)
    os.environ["DIPS_CALLBACK_STRIPED"] = "0"
    for win in (1, 3, 5, 11):
        res, last = {}, {}
        for rnd in range(2):
            for defer in (("1", "0") if rnd == 0 else ("0", "1")):
                os.environ["DIPS_DEFER_UPLOAD"] = defer
                cs = ComputeState(False, win, 5.0, DiPsFilter.Unfiltered, ChromaFilter.None_)
                lib, hd = cs._hd._lib, cs._hd
                for t in range(8):
                    hd.check(lib.dips_frame_callback(hd.ptr, W, H, host[t].ctypes.data, host[t].nbytes,
                                                     out.ctypes.data, out.nbytes))
                t0 = time.perf_counter()
                for t in range(8, F):
                    hd.check(lib.dips_frame_callback(hd.ptr, W, H, host[t].ctypes.data, host[t].nbytes,
                                                     out.ctypes.data, out.nbytes))
                dt = time.perf_counter() - t0
                cs.close()
                res.setdefault(defer, []).append((F - 8) / dt)
                last[defer] = out.copy()
        print(json.dumps({"window": win, "deferred_fps": [round(v, 1) for v in res["1"]],
                          "dma_fps": [round(v, 1) for v in res["0"]],
                          "outputs_equal": bool(np.array_equal(last["1"], last["0"]))}), flush=True)
    for k in ("DIPS_CALLBACK_STRIPED", "DIPS_DEFER_UPLOAD"):
        os.environ.pop(k, None)
    # dips_alt send_frame with a window: zero-copy (default) vs DMA
    from dips_amd.alt import DiPsCompute, DiPsProperties
    for win in (3, 5, 11):
        res, last = {}, {}
        for rnd in range(2):
            for direct in (("1", "0") if rnd == 0 else ("0", "1")):
                os.environ["DIPS_CALLBACK_DIRECT"] = direct
                c = DiPsCompute(2, H, W, DiPsProperties(window_size=win))
                ha = c._host
                for t in range(4):
                    ha.check(ha._lib.dips_alt_send_frame(ha.ptr, host[t].ctypes.data, host[t].nbytes, 0,
                                                         out.ctypes.data, out.nbytes))
                t0 = time.perf_counter()
                for t in range(4, F):
                    ha.check(ha._lib.dips_alt_send_frame(ha.ptr, host[t].ctypes.data, host[t].nbytes, 0,
                                                         out.ctypes.data, out.nbytes))
                dt = time.perf_counter() - t0
                c.close()
                res.setdefault(direct, []).append((F - 4) / dt)
                last[direct] = out.copy()
        print(json.dumps({"alt_window": win, "zero_copy_fps": [round(v, 1) for v in res["1"]],
                          "dma_fps": [round(v, 1) for v in res["0"]],
                          "outputs_equal": bool(np.array_equal(last["1"], last["0"]))}), flush=True)
    os.environ.pop("DIPS_CALLBACK_DIRECT", None)


if __name__ == "__main__":
    main()
