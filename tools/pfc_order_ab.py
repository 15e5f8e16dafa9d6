#!/usr/bin/env python3
"""pfc_order_ab.py -- the per-frame call's copy-pool order (host_stream.h
direct_interleave): DIPS_DIRECT_ORDER=0 (every staging piece, then the
copy-outs) against the interleaved default (a stripe's keys expanded as soon
as its kernel has finished, beside the packing of later stripes).  The bench
leg's loop (dips_frame_callback on 4K RGBA8 from pageable memory, each output
into its own pre-faulted buffer, every output compared with the batch path
after the loop), the two orders alternated over rounds in ONE process; plus
dips_alt send_frame the same way.  Run on the GPU box:
python tools/pfc_order_ab.py [rounds] [frames]"""
from __future__ import annotations

import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 4
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 208
    import torch
    from dips_amd import ChromaFilter, ComputeState, DiffSeriesOperator, DiPsFilter, PixelFormat
    W, H, warm = 3840, 2160, 8
    gen = DiffSeriesOperator(PixelFormat.RGBA8)
    dev = torch.empty((n, H, W, 4), dtype=torch.uint8, device="cuda")
    gen.synth_device(dev, W, H, 0xD1B5 ^ 0x4A, 0)
    gen.close()
    host = dev.cpu().numpy()
    wants = {}
    for colorize in (False, True):
        b = ComputeState(colorize, 1, 5.0, DiPsFilter.Unfiltered, ChromaFilter.None_)
        od = torch.empty_like(dev)
        b.frame_callback_batch_device(dev, od)
        torch.cuda.synchronize()
        wants[colorize] = od.cpu().numpy()
        b.close()
        del od
    del dev
    torch.cuda.empty_cache()
    outs = np.empty_like(host)
    outs.fill(0)
    for r in range(rounds):
        for order in (("1", "0") if r % 2 == 0 else ("0", "1")):
            for colorize in (False, True):
                os.environ["DIPS_DIRECT_ORDER"] = order
                cs = ComputeState(colorize, 1, 5.0, DiPsFilter.Unfiltered, ChromaFilter.None_)
                lib, hd = cs._hd._lib, cs._hd
                times = []
                for t in range(n):
                    t0 = time.perf_counter()
                    hd.check(lib.dips_frame_callback(hd.ptr, W, H, host[t].ctypes.data, host[t].nbytes,
                                                     outs[t].ctypes.data, outs[t].nbytes))
                    if t >= warm:
                        times.append(time.perf_counter() - t0)
                cs.close()
                ok = bool(np.array_equal(outs, wants[colorize]))
                print(json.dumps({"round": r, "order": "interleaved" if order == "1" else "staging first",
                                  "colorize": colorize, "frames_per_s": round(len(times) / sum(times), 1),
                                  "median_ms": round(float(np.median(times)) * 1e3, 4), "equal": ok}), flush=True)
    os.environ.pop("DIPS_DIRECT_ORDER", None)


if __name__ == "__main__":
    main()
