#!/usr/bin/env python3
"""nt_copy_ab.py -- in-process A/B of a host-path switch, alternated over
rounds, on every host-memory path of the library.  Default: the staging copy
(copy_pool.h host_copy: streaming AVX2 stores vs memcpy, DIPS_NT_COPY=1/0);
--var DIPS_PIPE_KERNEL_COPY: the host-fed pipelines' chunk copies by kernel
vs DMA engine (host_stream.h pipe_h2d / pipe_d2h).  Paths:
  * dips frame_callback, one 4K RGBA8 frame per call (the reference's own
    pattern, dips/src/lib.rs:233-246), striped;
  * dips_alt send_frame, one frame per call;
  * dips frame_callback_batch from pageable host frames (pipelined chunks);
  * the series from pageable host frames (dips_diff_series_streamed), 4K RGB8.
Outputs are checked equal between the two copies.  One JSON line per
(path, copy, round) and a summary line per path."""
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
    from dips_amd import ChromaFilter, ComputeState, DiffSeriesOperator, DiPsFilter, Mode, PixelFormat
    from dips_amd.alt import DiPsCompute

    import argparse
    ap = argparse.ArgumentParser()
    ap.add_argument("frames", type=int, nargs="?", default=48)
    ap.add_argument("rounds", type=int, nargs="?", default=3)
    ap.add_argument("--var", default="DIPS_NT_COPY")
    ap.add_argument("--values", default="1,0", help="values of --var, alternated (first two summarised as on/off)")
    args = ap.parse_args()
    values = args.values.split(",")
    W, H = 3840, 2160
    F, rounds, var = args.frames, args.rounds, args.var
    dev = torch.empty((F, H, W, 4), dtype=torch.uint8, device="cuda")
    op = DiffSeriesOperator(PixelFormat.RGBA8)
    op.synth_device(dev, W, H, 0xD1B5, 0)
    op.close()
    host = dev.cpu().numpy()
    del dev
    dev3 = torch.empty((96, H, W, 3), dtype=torch.uint8, device="cuda")
    op3 = DiffSeriesOperator(PixelFormat.RGB8, Mode.PerFrame, 8 / 255)
    op3.synth_device(dev3, W, H, 0xD1B5, 0)
    host3 = dev3.cpu().numpy()
    del dev3
    fb = W * H * 4
    out = np.zeros((H, W, 4), dtype=np.uint8)
    outs = np.zeros_like(host)

    cs = ComputeState(False, 1, 5.0, DiPsFilter.Unfiltered, ChromaFilter.None_)
    lib, hd = cs._hd._lib, cs._hd
    for t in range(8):
        hd.check(lib.dips_frame_callback(hd.ptr, W, H, host[t].ctypes.data, host[t].nbytes, out.ctypes.data, out.nbytes))
    alt = DiPsCompute(2, H, W)
    ha = alt._host
    for t in range(4):
        ha.check(ha._lib.dips_alt_send_frame(ha.ptr, host[t].ctypes.data, host[t].nbytes, 0, out.ctypes.data, out.nbytes))
    csb = ComputeState(False, 1, 5.0, DiPsFilter.Unfiltered, ChromaFilter.None_)
    hb = csb._hd
    hb.check(hb._lib.dips_frame_callback_batch(hb.ptr, W, H, host[:8].ctypes.data, 8, outs.ctypes.data))
    op3.streamed(host3[:16], chunk_frames=8)

    def callback():
        t0 = time.perf_counter()
        for t in range(8, F):
            hd.check(lib.dips_frame_callback(hd.ptr, W, H, host[t].ctypes.data, host[t].nbytes,
                                             out.ctypes.data, out.nbytes))
        return F - 8, time.perf_counter() - t0, int(out[::97, ::89].astype(np.uint64).sum())

    def send_frame():
        t0 = time.perf_counter()
        for t in range(4, F):
            ha.check(ha._lib.dips_alt_send_frame(ha.ptr, host[t].ctypes.data, host[t].nbytes, 0,
                                                 out.ctypes.data, out.nbytes))
        return F - 4, time.perf_counter() - t0, int(out[::97, ::89].astype(np.uint64).sum())

    def batch():
        t0 = time.perf_counter()
        hb.check(hb._lib.dips_frame_callback_batch(hb.ptr, W, H, host.ctypes.data, F, outs.ctypes.data))
        return F, time.perf_counter() - t0, int(outs[:, ::97, ::89].astype(np.uint64).sum())

    def streamed():
        t0 = time.perf_counter()
        s = op3.streamed(host3, chunk_frames=8)
        return host3.shape[0], time.perf_counter() - t0, int(s.as_array().astype(np.uint64).sum() % (1 << 62))

    paths = [("frame_callback per frame (striped), 4K RGBA8", callback, 2 * fb),
             ("dips_alt send_frame per frame, 4K RGBA8", send_frame, 2 * fb),
             ("frame_callback_batch from host, 4K RGBA8", batch, 2 * fb),
             ("series streamed from host, 4K RGB8", streamed, W * H * 3)]
    summary = {p[0]: {**{v: [] for v in values}, "check": {}} for p in paths}
    for rnd in range(rounds):
        for nt in (values if rnd % 2 == 0 else values[::-1]):
            os.environ[var] = nt
            for name, fn, bpf in paths:
                n, dt, chk = fn()
                fps = n / dt
                summary[name][nt].append(fps)
                if rnd >= 1:  # round 0's batch follows the warm-up frames, later ones the same tail
                    summary[name]["check"].setdefault(nt, chk)
                print(json.dumps({"path": name, var: nt, "round": rnd, "frames": n,
                                  "frames_per_s": round(fps, 1), "ms_per_frame": round(dt / n * 1e3, 3),
                                  "pcie_GBps": round(n * bpf / dt / 1e9, 2), "check": chk}), flush=True)
    os.environ.pop(var, None)
    for name, s in summary.items():
        print(json.dumps({"path": name, "summary": True, "var": var,
                          "fps_median": {v: round(float(np.median(s[v])), 1) for v in values},
                          "ratio_first_second": round(float(np.median(s[values[0]]) / np.median(s[values[1]])), 4),
                          "outputs_equal": len(set(s["check"].values())) == 1}), flush=True)
    for o in (cs, csb, alt):
        o.close()
    op3.close()


if __name__ == "__main__":
    main()
