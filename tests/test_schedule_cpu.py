"""The part-major schedule restatement used by the GPU tests (tests/_sched.py)
against the figures dips_abi.hip part_geometry documents: the bench's 4K
batch, the 1080p part-major parity shape, and the shapes the new GPU tests
rely on (256-CU MI355X; the RGB8 kernel's 5 vecs per lane run 4 waves per
SIMD)."""
from _sched import part_schedule

CUS = 256


def _tiles(w, h, c=3, unroll=5):
    return (w * h // 4 + 64 * unroll - 1) // (64 * unroll)


def test_bench_batch_schedule():
    # 3840x2160 RGB8, 5000 frames, 4 waves/SIMD: L = 1000, 4,050 waves
    # (32,400 items in 8 rounds)
    assert part_schedule(_tiles(3840, 2160), 5000, 4 * 4 * CUS) == (1000, 5, 4050)


def test_parity_shape_schedule():
    # tests/test_gpu_series.py: 1080p RGB8 523 frames -> 4 parts of 131
    L, parts, _ = part_schedule(_tiles(1920, 1080), 523, 4 * 4 * CUS)
    assert (L, parts) == (131, 4)


def test_rehearsal_and_timed_shapes_take_part_major():
    # bench.py at N > 1 caps 4 waves/SIMD; a rank's (F - 1)-frame launch
    L, parts, waves = part_schedule(_tiles(2560, 1440), 299, 4 * 4 * CUS)
    assert (L, parts) == (150, 2) and waves == 2880
    # the timed configuration's 520-frame parity batch
    L, parts, _ = part_schedule(_tiles(3840, 2160), 520, 4 * 4 * CUS)
    assert (L, parts) == (174, 3)


def test_short_batches_keep_contiguous_ranges():
    assert part_schedule(_tiles(3840, 2160), 255, 4 * 4 * CUS) is None
    # 640x360: too few tiles for >= 128-frame parts to fill the slots
    assert part_schedule(_tiles(640, 360), 299, 4 * 4 * CUS) is None
