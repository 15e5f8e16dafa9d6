"""tools/placement.py resident_frames (bench.py's batch allocation): the
batch lands in the plain allocation unless the second candidate is faster by
more than the threshold, holds the frames the fill wrote, the other
candidate is released, and the report carries both candidates' times and the
margin; probe=False and a batch too large for two candidates give one plain
allocation."""
import numpy as np
import pytest

from oracle import oracle

pytestmark = pytest.mark.gpu

W, H, C, F = 640, 360, 3, 40
TAU = 8 / 255


def test_resident_frames_probe_and_plain():
    import torch
    from dips_amd import DiffSeriesOperator, Mode, PixelFormat
    from tools.placement import choose, resident_frames
    dev = torch.device("cuda", 0)
    op = DiffSeriesOperator(PixelFormat.RGB8, Mode.PerFrame, TAU, time_kernel=True)
    try:
        fill = lambda t: op.synth_device(t, W, H, 0xD1B5, 0)  # noqa: E731
        torch.cuda.synchronize()
        t, rep = resident_frames(op, (F, H, W, C), dev, fill)
        assert rep["probe"] and rep["kept"] in (0, 1) and len(rep["candidate_kernel_ms"]) == 2
        ms = rep["candidate_kernel_ms"]
        assert rep["kept"] == choose(ms[0], ms[1], rep["threshold"])[0]
        # the kept buffer holds the synthesised frames; the series matches the oracle
        want_frames = torch.empty_like(t)
        fill(want_frames)
        assert torch.equal(t, want_frames)
        ser = torch.zeros((F, 4), dtype=torch.int64, device=dev)
        op.run_device(t, ser)
        torch.cuda.synchronize()
        want, _, _ = oracle.series(t.cpu().numpy(), mode=1, tau=TAU)
        assert np.array_equal(ser.cpu().numpy().view(np.uint64), want)
        # the timer was left reset for the caller
        assert op.kernel_time()[1] == 1
        p, rep2 = resident_frames(op, (F, H, W, C), dev, fill, probe=False)
        assert rep2 == {"probe": False, "reason": "disabled"} and torch.equal(p, want_frames)
        # no room for two candidates: one plain allocation
        free, _ = torch.cuda.mem_get_info(dev)
        big = (int(free * 0.6) // (H * W * C), H, W, C)
        q, rep3 = resident_frames(op, big, dev, lambda x: None)
        assert rep3 == {"probe": False, "reason": "no room for two candidates"} and tuple(q.shape) == big
        del q
        torch.cuda.empty_cache()
    finally:
        op.close()
