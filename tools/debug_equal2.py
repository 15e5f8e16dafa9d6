import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from dips_amd import DiffSeriesOperator, Mode, PixelFormat
W, H, SEED = 3840, 2160, 0xD1B5
op = DiffSeriesOperator(PixelFormat.RGB8, Mode.PerFrame, 8 / 255)
for F in (8, 80, 170, 180, 400, 5000):
    fr = torch.empty((F, H, W, 3), dtype=torch.uint8, device="cuda")
    op.synth_device(fr, W, H, SEED, 0)
    buf = torch.empty((2, H, W, 3), dtype=torch.uint8, device="cuda")
    op.synth_device(buf, W, H, SEED, 0)
    torch.cuda.synchronize()
    a, b = buf[1], fr[1]
    ne = int((a != b).sum())
    print(F, "torch.equal", torch.equal(a, b), "ne.sum", ne, "cpu equal", torch.equal(a.cpu(), b.cpu()),
          "clone", torch.equal(a, b.clone()), "eq.all", bool((a == b).all()), flush=True)
    del fr, buf
    torch.cuda.empty_cache()
op.close()
