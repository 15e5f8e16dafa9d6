#!/usr/bin/env python3
"""callback_direct_ab.py -- one 4K RGBA8 frame per dips_frame_callback call
(the reference's own pattern, dips/src/lib.rs:233-246), the zero-copy form
(DIPS_CALLBACK_DIRECT=1: the main kernel reads the staged frame from and
writes its output to pinned host memory over PCIe) against the DMA form
(=0: hipMemcpyAsync stripes up and down), alternated in one process, for
several stripe sizes (DIPS_PIECE_BYTES).  Every output of both forms is
compared with the plain add_texture + dispatch sequence's."""
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
    rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    dev = torch.empty((F, H, W, 4), dtype=torch.uint8, device="cuda")
    op = DiffSeriesOperator(PixelFormat.RGBA8)
    op.synth_device(dev, W, H, 0xD1B5, 0)
    op.close()
    host = dev.cpu().numpy()
    del dev
    out = np.zeros((H, W, 4), dtype=np.uint8)

    # reference outputs: the plain add_texture + dispatch sequence, frames 0..F-1 then 8..F-1 again
    ref = ComputeState(False, 1, 5.0, DiPsFilter.Unfiltered, ChromaFilter.None_)
    rl, rh = ref._hd._lib, ref._hd
    os.environ["DIPS_CALLBACK_STRIPED"] = "0"
    os.environ["DIPS_DEFER_UPLOAD"] = "0"  # the reference pass: DMA upload + DMA readback
    want = {}
    for t in list(range(F)) + list(range(8, F)):
        rh.check(rl.dips_frame_callback(rh.ptr, W, H, host[t].ctypes.data, host[t].nbytes, out.ctypes.data, out.nbytes))
        if t >= 8:
            want[t] = out.copy()
    os.environ.pop("DIPS_CALLBACK_STRIPED")
    os.environ.pop("DIPS_DEFER_UPLOAD")
    ref.close()

    cs = ComputeState(False, 1, 5.0, DiPsFilter.Unfiltered, ChromaFilter.None_)
    lib, hd = cs._hd._lib, cs._hd
    for t in range(F):  # the same stream prefix as the reference pass: every timed pass follows frames F-3..F-1
        hd.check(lib.dips_frame_callback(hd.ptr, W, H, host[t].ctypes.data, host[t].nbytes, out.ctypes.data, out.nbytes))
    # (name, DIPS_CALLBACK_DIRECT, stripe bytes, extra env): the direct form
    # puts odd stripes on a second stream (DIPS_DIRECT_STREAMS=1: all on one)
    # and cuts each stripe into DIPS_DIRECT_SPLIT copy-pool pieces
    variants = [("dma", "0", 4 << 20, {}),
                ("direct split1 full-first", "1", 4 << 20, {"DIPS_DIRECT_SPLIT": "1", "DIPS_DIRECT_FIRST": "0"}),
                ("direct split8 full-first", "1", 4 << 20, {"DIPS_DIRECT_SPLIT": "8", "DIPS_DIRECT_FIRST": "0"}),
                ("direct split8", "1", 4 << 20, {"DIPS_DIRECT_SPLIT": "8"}),
                ("direct split16", "1", 4 << 20, {"DIPS_DIRECT_SPLIT": "16"}),
                ("direct split8", "1", 8 << 20, {"DIPS_DIRECT_SPLIT": "8"}),
                # the reference's own sequence, add_texture + dispatch (the
                # unstriped frame_callback): staged frame read by the dispatch
                # (deferred upload) or DMA up + DMA down
                ("add_texture+dispatch deferred", "1", 4 << 20, {"DIPS_CALLBACK_STRIPED": "0", "DIPS_DEFER_UPLOAD": "1"}),
                ("add_texture+dispatch dma", "1", 4 << 20, {"DIPS_CALLBACK_STRIPED": "0", "DIPS_DEFER_UPLOAD": "0"})]
    res = {}
    for rnd in range(rounds):
        for name, direct, piece, extra in (variants if rnd % 2 == 0 else variants[::-1]):
            os.environ["DIPS_CALLBACK_DIRECT"] = direct
            os.environ["DIPS_PIECE_BYTES"] = str(piece)
            for k in ("DIPS_DIRECT_STREAMS", "DIPS_DIRECT_SPLIT", "DIPS_DIRECT_FIRST", "DIPS_CALLBACK_STRIPED",
                      "DIPS_DEFER_UPLOAD"):
                os.environ.pop(k, None)
            os.environ.update(extra)
            ok = True
            dt = 0.0
            for t in range(8, F):
                t0 = time.perf_counter()
                hd.check(lib.dips_frame_callback(hd.ptr, W, H, host[t].ctypes.data, host[t].nbytes,
                                                 out.ctypes.data, out.nbytes))
                dt += time.perf_counter() - t0
                if t in (8, F // 2, F - 1):  # spot checks (outside the timed calls)
                    ok = ok and bool(np.array_equal(out, want[t]))
            key = f"{name} {piece >> 20} MiB"
            res.setdefault(key, []).append((F - 8) / dt)
            print(json.dumps({"variant": key, "round": rnd, "frames_per_s": round((F - 8) / dt, 1),
                              "ms_per_frame": round(dt / (F - 8) * 1e3, 3),
                              "pcie_GBps_each_way": round((F - 8) * W * H * 4 / dt / 1e9, 2),
                              "outputs_equal_plain": ok}), flush=True)
    for k in ("DIPS_CALLBACK_DIRECT", "DIPS_PIECE_BYTES", "DIPS_DIRECT_STREAMS", "DIPS_DIRECT_SPLIT",
              "DIPS_DIRECT_FIRST", "DIPS_CALLBACK_STRIPED", "DIPS_DEFER_UPLOAD"):
        os.environ.pop(k, None)
    cs.close()
    # dips_alt send_frame, one frame per call, both forms (default N = 2)
    from dips_amd.alt import DiPsCompute
    c = DiPsCompute(2, H, W)
    ha = c._host
    for t in range(F):
        ha.check(ha._lib.dips_alt_send_frame(ha.ptr, host[t].ctypes.data, host[t].nbytes, 0, out.ctypes.data, out.nbytes))
    last = {}
    for rnd in range(rounds):
        for name, direct in (("alt dma", "0"), ("alt direct", "1")) if rnd % 2 == 0 else (("alt direct", "1"), ("alt dma", "0")):
            os.environ["DIPS_CALLBACK_DIRECT"] = direct
            os.environ["DIPS_PIECE_BYTES"] = str(4 << 20)
            t0 = time.perf_counter()
            for t in range(8, F):
                ha.check(ha._lib.dips_alt_send_frame(ha.ptr, host[t].ctypes.data, host[t].nbytes, 0,
                                                     out.ctypes.data, out.nbytes))
            dt = time.perf_counter() - t0
            last.setdefault(name, out.copy())
            res.setdefault(name + " 4 MiB", []).append((F - 8) / dt)
            print(json.dumps({"variant": name + " 4 MiB", "round": rnd, "frames_per_s": round((F - 8) / dt, 1),
                              "ms_per_frame": round(dt / (F - 8) * 1e3, 3),
                              "pcie_GBps_each_way": round((F - 8) * W * H * 4 / dt / 1e9, 2),
                              "outputs_equal_other_form": bool(len(last) < 2 or np.array_equal(*last.values()))}),
                  flush=True)
    c.close()
    for k in ("DIPS_CALLBACK_DIRECT", "DIPS_PIECE_BYTES"):
        os.environ.pop(k, None)
    for k, v in res.items():
        print(json.dumps({"variant": k, "summary": True, "median_frames_per_s": round(float(np.median(v)), 1)}),
              flush=True)


if __name__ == "__main__":
    main()
