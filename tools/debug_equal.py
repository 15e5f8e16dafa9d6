import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from dips_amd import DiffSeriesOperator, Mode, PixelFormat
W, H, SEED = 3840, 2160, 0xD1B5
op = DiffSeriesOperator(PixelFormat.RGB8, Mode.PerFrame, 8 / 255)
for (w, h) in [(256, 96), (3840, 2160)]:
    fr = torch.empty((8, h, w, 3), dtype=torch.uint8, device="cuda")
    op.synth_device(fr, w, h, SEED, 0)
    buf = torch.empty((2, h, w, 3), dtype=torch.uint8, device="cuda")
    op.synth_device(buf, w, h, SEED, 3)
    torch.cuda.synchronize()
    a, b = buf[1], fr[4]
    print(w, h, "torch.equal", torch.equal(a, b), "ne.any", bool((a != b).any()), "ne.sum", int((a != b).sum()),
          "cpu equal", torch.equal(a.cpu(), b.cpu()), "flat", torch.equal(a.reshape(-1), b.reshape(-1)),
          "clone", torch.equal(a.clone(), b.clone()), "int16", torch.equal(a.to(torch.int16), b.to(torch.int16)),
          flush=True)
    x = torch.zeros(w * h * 3, dtype=torch.uint8, device="cuda")
    y = torch.zeros(w * h * 3, dtype=torch.uint8, device="cuda")
    print("zeros equal", torch.equal(x, y), "small zeros", torch.equal(x[:1000], y[:1000]), flush=True)
op.close()
