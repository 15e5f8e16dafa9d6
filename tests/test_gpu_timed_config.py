"""The exact configuration bench.py times, pinned to the oracle frame by
frame (BASELINE.json configs[2]: 3840x2160 RGB8, 'per-frame', tau = 8/255,
the default intensity-sum form ISI = 1 -- series_v2_kernel<3, 0, 5, true,
false, false, 1>).

The bench's 5000-frame batch runs the part-major schedule (series_abi.hip
part_geometry: 5 parts of 1000 frames); a 520-frame batch of the same frames
runs it with 3 parts of 174 frames (the last 172) on a 256-CU MI355X, so
items start mid-batch and the last part is short -- asserted through the
library's own geometry, then every one of the 520 series entries must equal
the oracle's (get_intensity, dips/src/gpu/shaders/dips_shader.wgsl:64-82).
Also at 4K: 'overall' (configs[3]'s mode, part-major since round 4) and
RGBA8 frames at a +2-byte offset (the aligned-load form a caller's ring
buffer lands on).

BASELINE.json configs[4] (7680x4320 RGB8, tau = 8/255: ISI = 1) on the
schedule its 1,250-frame-per-GPU batch runs: 260 frames take the part-major
schedule with 2 parts (asserted through the library's geometry, both modes),
and every series entry must equal the oracle's."""
import numpy as np
import pytest

from oracle import oracle
from _sched import library_schedule

pytestmark = pytest.mark.gpu

W, H, SEED, TAU = 3840, 2160, 0xD1B5, 8.0 / 255.0


def _series_vs_oracle(fmt_name, mode, n, offset=0, t0=0, W=W, H=H, schedule=None):
    import torch
    from dips_amd import DiffSeriesOperator, Mode, PixelFormat
    fmt = getattr(PixelFormat, fmt_name)
    c = int(fmt)
    fb = W * H * c
    op = DiffSeriesOperator(fmt, Mode(mode), TAU, 0)
    try:
        if schedule is None:
            schedule = mode == 1 and offset == 0
        sch = library_schedule(op, W, H, n) if schedule else None
        buf = torch.empty(n * fb + 16, dtype=torch.uint8, device="cuda")
        dev = buf[offset:offset + n * fb].view(n, H, W, c)
        op.synth_device(dev, W, H, SEED, t0)
        ser = torch.zeros((n, 4), dtype=torch.int64, device="cuda")
        op.run_device(dev, ser)
        torch.cuda.synchronize()
        got = ser.cpu().numpy().view(np.uint64)
        frames = dev.cpu().numpy()
        del buf, dev
        torch.cuda.empty_cache()
    finally:
        op.close()
    out4, _, _ = oracle.series(frames, mode=mode, tau=TAU, nthreads=16)
    bad = np.nonzero(~np.all(got == out4, axis=1))[0]
    assert bad.size == 0, f"{fmt_name} mode {mode} +{offset}: frames differing from the oracle: {bad[:10]}"
    return sch


@pytest.mark.timeout(600)
def test_timed_config_per_frame_part_major_every_frame(monkeypatch):
    monkeypatch.delenv("DIPS_SERIES_WAVES_PER_SIMD", raising=False)
    sch = _series_vs_oracle("RGB8", 1, 520)
    assert sch is not None and sch[1] >= 3, sch  # part-major, >= 3 parts


@pytest.mark.timeout(600)
def test_timed_config_overall_every_frame():
    _series_vs_oracle("RGB8", 0, 300, t0=17)


@pytest.mark.timeout(600)
def test_timed_config_rgba8_offset2_every_frame():
    _series_vs_oracle("RGBA8", 1, 300, offset=2, t0=5)


@pytest.mark.timeout(1200)
@pytest.mark.parametrize("mode", [0, 1])
def test_configs4_8k_part_major_every_frame(monkeypatch, mode):
    """configs[4]: 7680x4320 RGB8, tau 8/255, 260 frames on the part-major
    schedule (>= 2 parts), every entry against the oracle (the bench's
    1,250-frame batch takes 3 parts of the same tiles)."""
    monkeypatch.delenv("DIPS_SERIES_WAVES_PER_SIMD", raising=False)
    sch = _series_vs_oracle("RGB8", mode, 260, t0=1000, W=7680, H=4320, schedule=True)
    assert sch is not None and sch[1] >= 2, sch
