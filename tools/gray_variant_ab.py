#!/usr/bin/env python3
"""gray_variant_ab.py -- in-process A/B of the GRAY8 table kernel's variants,
read per call: vecs per lane of the layout-2 table (a number: DIPS_GRAY_LUT_U),
arithmetic vecs and waves per group ("a<NA>w<W>": DIPS_GRAY_ALU /
DIPS_GRAY_ALU_WAVES) or the table layout ("L3", "L2", "L3u3": DIPS_GRAY_LUT,
U = 4 or the number after u; a trailing "c": DIPS_SERIES_PARTS=0, the
contiguous ranges instead of the part-major schedule);
one batch of 4K gray8 frames, per-frame, tau 8/255; variants alternated over
rounds, kernel time by hipEvents, series compared with the first variant's.
Run on the GPU box: python tools/gray_variant_ab.py [rounds] [frames] [variants] [pf|overall] [map|nomap]
[synth|random] (with the map, GBps counts the map's writes too; "random":
i.i.d. uniform frames instead of the bench's synthetic clip).
"""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 6000
    variants = (sys.argv[3] if len(sys.argv) > 3 else "4,2,3").split(",")
    mode = sys.argv[4] if len(sys.argv) > 4 else "pf"
    with_map = len(sys.argv) > 5 and sys.argv[5] == "map"
    content = sys.argv[6] if len(sys.argv) > 6 else "synth"
    import torch
    from dips_amd import DiffSeriesOperator, Mode, PixelFormat
    W, H = 3840, 2160
    op = DiffSeriesOperator(PixelFormat.Gray8, Mode.PerFrame if mode == "pf" else Mode.Overall, 8.0 / 255.0,
                            time_kernel=True)
    frames = torch.empty((n, H, W), dtype=torch.uint8, device="cuda")
    dmap = torch.empty_like(frames) if with_map else None
    if content == "random":
        g = torch.Generator(device="cuda")
        g.manual_seed(7)
        for k in range(0, n, 500):
            frames[k:k + 500].copy_(torch.randint(0, 256, frames[k:k + 500].shape, dtype=torch.uint8,
                                                  device="cuda", generator=g))
    else:
        op.synth_device(frames, W, H, 0xD1B5, 0)
    ser = torch.zeros((n, 4), dtype=torch.int64, device="cuda")
    ref = None
    for r in range(rounds):
        for v in variants:
            name = v
            os.environ.pop("DIPS_SERIES_PARTS", None)
            if v.endswith("c"):  # ...c: contiguous ranges instead of the part-major schedule
                os.environ["DIPS_SERIES_PARTS"] = "0"
                v = v[:-1]
            if v.startswith("L"):  # L<layout>[u<U>]
                lay, _, u = v[1:].partition("u")
                os.environ["DIPS_GRAY_LUT"] = lay
                os.environ["DIPS_GRAY_ALU"] = "0"
                os.environ["DIPS_GRAY_LUT_U"] = u or "4"
            elif v.startswith("a"):
                os.environ["DIPS_GRAY_LUT"] = "2"
                na, w = v[1:].split("w")
                os.environ["DIPS_GRAY_ALU"], os.environ["DIPS_GRAY_ALU_WAVES"] = na, w
                os.environ["DIPS_GRAY_LUT_U"] = "4"
            else:
                os.environ["DIPS_GRAY_LUT"] = "2"
                os.environ["DIPS_GRAY_ALU"] = "0"
                os.environ["DIPS_GRAY_LUT_U"] = v
            op.run_device(frames, ser, map_out=dmap)
            torch.cuda.synchronize()
            op.kernel_time(reset=True)
            for _ in range(5):
                op.run_device(frames, ser, map_out=dmap)
            torch.cuda.synchronize()
            ms = float(np.median(op.kernel_times()))
            h = ser.cpu().numpy()
            if ref is None:
                ref = h
            gbs = n * W * H * (2 if with_map else 1) / (ms / 1e3) / 1e9
            print(json.dumps({"round": r, "variant": name, "mode": mode, "map": with_map, "content": content, "kernel_ms": round(ms, 4), "GBps": round(gbs, 1),
                              "frac_of_8TBps": round(gbs / 8000, 4), "series_equal_first": bool(np.array_equal(h, ref))}),
                  flush=True)
    op.close()


if __name__ == "__main__":
    main()
