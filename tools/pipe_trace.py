"""pipe_trace.py -- where the host-feed time of the dips_alt run loop goes:
the same sequence as host_feed_rate.py with Python-side phases timed."""
import sys, time
sys.path.insert(0, '/root/repo')
import numpy as np, torch
from dips_amd import DiffSeriesOperator, PixelFormat, ComputeState, DiPsFilter, ChromaFilter
from dips_amd.alt import DiPsRunner, _frames_u8
W, H = 3840, 2160
F = int(sys.argv[1]) if len(sys.argv) > 1 else 160
dev = torch.empty((F, H, W, 4), dtype=torch.uint8, device="cuda")
op = DiffSeriesOperator(PixelFormat.RGBA8); op.synth_device(dev, W, H, 0xD1B5, 0); op.close()
host = dev.cpu().numpy(); del dev
cs = ComputeState(False, 1, 5.0, DiPsFilter.Unfiltered, ChromaFilter.None_)
cs.frame_callback_batch(W, H, host[:16]); t = time.perf_counter(); o = cs.frame_callback_batch(W, H, host)
print(f"compat {F/(time.perf_counter()-t):.1f} fps", flush=True); cs.close(); o = None
r = DiPsRunner(H, W); r(host[:16])
c = r.compute
for rep in range(3):
    t0 = time.perf_counter(); a = _frames_u8(host, c.rows, c.cols)
    t1 = time.perf_counter(); out = np.empty_like(a)
    t2 = time.perf_counter()
    h = c._host
    h.check(h._lib.dips_alt_run(h.ptr, a.ctypes.data, a.shape[0], None, 0, out.ctypes.data))
    t3 = time.perf_counter()
    out = None
    t4 = time.perf_counter()
    print(f"rep {rep}: frames_u8 {1e3*(t1-t0):.2f} empty {1e3*(t2-t1):.2f} run {1e3*(t3-t2):.2f} free {1e3*(t4-t3):.2f} ms -> {F/(t3-t0):.1f} fps", flush=True)
r.close()
