"""Test helper: the part-major schedule the library picks for a 'per-frame'
RGB8 / RGBA8 batch, restated from series_abi.hip part_geometry so that a test
can assert which schedule a launch runs (and that the library agrees: the
wave count it reports must equal the restatement's)."""
from __future__ import annotations


def resident_waves(op, width: int, height: int, n_frames: int) -> int:
    """Wave slots of the series kernel for this shape: the library's wave
    count for a batch of < 256 frames (the contiguous ranges, part_geometry
    starts at 256) that has more items than slots."""
    waves, tiles, _ = op.geometry(width, height, min(n_frames, 255))
    assert tiles * min(n_frames, 255) > waves, "batch too small to fill the wave slots"
    return int(waves)


def part_schedule(n_tiles: int, n_frames: int, resident: int):
    """(part_frames L, parts, n_waves) of part_geometry, or None when the
    batch keeps the contiguous ranges."""
    if n_frames < 256 or n_tiles == 0 or resident == 0:
        return None
    p_min = max((resident + n_tiles - 1) // n_tiles, (n_frames + 1249) // 1250)
    p_max = min(4 * p_min, n_frames // 128)
    if p_max < p_min:
        return None
    best_p, best_fill = 0, -1.0
    for p in range(p_min, p_max + 1):
        L = (n_frames + p - 1) // p
        parts = (n_frames + L - 1) // L
        items = parts * n_tiles
        k = (items + resident - 1) // resident
        fill = items / (k * resident)
        if fill > best_fill + 1e-9:
            best_fill, best_p = fill, p
        if fill >= 0.98:
            break
    L = (n_frames + best_p - 1) // best_p
    parts = (n_frames + L - 1) // L
    items = parts * n_tiles
    k = (items + resident - 1) // resident
    return L, parts, (items + k - 1) // k


def library_schedule(op, width: int, height: int, n_frames: int):
    """The restated schedule of a per-frame launch of n_frames, checked
    against the wave count the library reports for it."""
    resident = resident_waves(op, width, height, n_frames)
    waves, tiles, _ = op.geometry(width, height, n_frames)
    sch = part_schedule(int(tiles), n_frames, resident)
    want = sch[2] if sch else min(int(tiles) * n_frames, resident)
    assert int(waves) == want, (waves, want, sch)
    return sch
