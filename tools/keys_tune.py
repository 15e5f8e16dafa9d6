#!/usr/bin/env python3
"""keys_tune.py -- stripe geometry of the keyed zero-copy per-frame call
(dips_frame_callback, 4K RGBA8, gray keys): DIPS_PIECE_BYTES (stripe size),
DIPS_DIRECT_SPLIT (copy-pool pieces per stripe) and DIPS_DIRECT_FIRST (a
quarter first stripe or a full one), alternated over rounds in one process;
outputs compared with the first variant's.  `keys_tune.py 16 trace`: the
DIPS_STRIPE_TRACE timeline of a few calls with the default geometry (stderr)."""
from __future__ import annotations

import itertools
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    trace = "trace" in sys.argv
    if trace:  # read once per process by the library: set before the first call
        os.environ["DIPS_STRIPE_TRACE"] = "1"
        sys.argv.remove("trace")
    import torch
    from dips_amd import ChromaFilter, ComputeState, DiffSeriesOperator, DiPsFilter, PixelFormat
    W, H = 3840, 2160
    F = int(sys.argv[1]) if len(sys.argv) > 1 else 40
    rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 2
    dev = torch.empty((F, H, W, 4), dtype=torch.uint8, device="cuda")
    op = DiffSeriesOperator(PixelFormat.RGBA8)
    op.synth_device(dev, W, H, 0xD1B5, 0)
    op.close()
    host = dev.cpu().numpy()
    del dev
    out = np.zeros((H, W, 4), dtype=np.uint8)
    cs = ComputeState(False, 1, 5.0, DiPsFilter.Unfiltered, ChromaFilter.None_)
    lib, hd = cs._hd._lib, cs._hd
    call = lambda t: hd.check(lib.dips_frame_callback(hd.ptr, W, H, host[t].ctypes.data, host[t].nbytes,  # noqa: E731
                                                      out.ctypes.data, out.nbytes))
    for t in range(8):
        call(t)
    if trace:
        for t in range(8, 14):
            call(t)
        cs.close()
        return
    variants = list(itertools.product([2 << 20, 4 << 20, 8 << 20], ["4", "8", "16"], ["1", "0"]))
    want, res = {}, {}
    for rnd in range(rounds):
        for piece, split, first in (variants if rnd % 2 == 0 else variants[::-1]):
            os.environ["DIPS_PIECE_BYTES"] = str(piece)
            os.environ["DIPS_DIRECT_SPLIT"] = split
            os.environ["DIPS_DIRECT_FIRST"] = first
            ok, dt = True, 0.0
            for pos, t in enumerate(list(range(F - 3, F)) + list(range(8, F))):
                t0 = time.perf_counter()
                call(t)
                dt += time.perf_counter() - t0
                if pos in (3, F - 6):
                    want.setdefault(pos, out.copy())
                    ok = ok and bool(np.array_equal(out, want[pos]))
            n = F - 8 + 3
            k = f"piece {piece >> 20} MiB split {split} first {'quarter' if first == '1' else 'full'}"
            res.setdefault(k, []).append(n / dt)
            print(json.dumps({"variant": k, "round": rnd, "frames_per_s": round(n / dt, 1),
                              "outputs_equal": ok}), flush=True)
    for k in ("DIPS_PIECE_BYTES", "DIPS_DIRECT_SPLIT", "DIPS_DIRECT_FIRST"):
        os.environ.pop(k, None)
    for k, v in sorted(res.items(), key=lambda kv: -float(np.median(kv[1]))):
        print(json.dumps({"variant": k, "summary": True, "median_frames_per_s": round(float(np.median(v)), 1)}),
              flush=True)
    cs.close()


if __name__ == "__main__":
    main()
