"""Which rows of a big resident batch differ from small launches over the
same synthetic frames (bench self-check diagnosis)."""
import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch
from dips_amd import DiffSeriesOperator, Mode, PixelFormat

W, H, SEED = 3840, 2160, 0xD1B5
F = int(sys.argv[1]) if len(sys.argv) > 1 else 5000
for mode in (Mode.PerFrame, Mode.Overall):
    op = DiffSeriesOperator(PixelFormat.RGB8, mode, 8 / 255, time_kernel=True)
    fr = torch.empty((F, H, W, 3), dtype=torch.uint8, device="cuda")
    op.synth_device(fr, W, H, SEED, 0)
    ser = torch.zeros((F, 4), dtype=torch.int64, device="cuda")
    op.run_device(fr, ser, ref=None if mode == Mode.PerFrame else fr[0])
    torch.cuda.synchronize()
    big = ser.cpu().numpy()
    for g in [0, 1, 2, 3, 100, 400, 600, 689, 1000, 1591, 3149, F - 1]:
        if g >= F:
            continue
        g0 = max(g - 1, 0)
        buf = torch.empty((2, H, W, 3), dtype=torch.uint8, device="cuda")
        op.synth_device(buf, W, H, SEED, g0)
        same_frames = bool(torch.equal(buf[1 if g > 0 else 0], fr[g]))
        out = torch.zeros((2, 4), dtype=torch.int64, device="cuda")
        if mode == Mode.PerFrame:
            op.run_device(buf, out)
        else:
            f0 = torch.empty((1, H, W, 3), dtype=torch.uint8, device="cuda")
            op.synth_device(f0, W, H, SEED, 0)
            op.run_device(buf, out, ref=f0[0])
            same_frames = same_frames and bool(torch.equal(f0[0], fr[0]))
        torch.cuda.synchronize()
        small = out.cpu().numpy()[1 if g > 0 else 0]
        # the same frames in the big buffer, 2-frame launch from a view
        out2 = torch.zeros((2, 4), dtype=torch.int64, device="cuda")
        op.run_device(fr[g0:g0 + 2], out2, ref=None if mode == Mode.PerFrame else fr[0])
        torch.cuda.synchronize()
        view = out2.cpu().numpy()[1 if g > 0 else 0]
        print(int(mode), g, "frames_equal", same_frames, "big", big[g].tolist(), "small", small.tolist(),
              "view", view.tolist(), flush=True)
    op.close()
    del fr, ser
    torch.cuda.empty_cache()
