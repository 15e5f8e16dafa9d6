"""CPU tests of the host-side mirror of the reference API (no GPU)."""
import numpy as np
import pytest

from dips_amd import (ChromaFilter, DiPsFilter, DiPsProperties, Mode, PixelFormat, Series,
                      si_from_fixed)
from dips_amd.api import _frame_geometry


def test_filter_codes_match_reference():
    """Into<f64> for DiPsFilter / ChromaFilter, dips/src/lib.rs:32-61."""
    assert int(DiPsFilter.Unfiltered) == 255
    assert int(DiPsFilter.Sigmoid) == 0
    assert int(DiPsFilter.InverseSigmoid) == 1
    assert [int(c) for c in (ChromaFilter.None_, ChromaFilter.Red, ChromaFilter.Green,
                             ChromaFilter.Blue)] == [0, 1, 2, 3]


def test_properties_builder_defaults_and_chaining():
    """DiPsProperties::new / builder / build, dips/src/lib.rs:63-170."""
    p = DiPsProperties.new()
    assert (p.colorize_, p.spatial_window_size_, p.sensitivity_) == (False, 1, 5.0)
    assert p.filter_type_ == DiPsFilter.Unfiltered and p.chroma_filter_ == ChromaFilter.None_
    assert p.get_video_path() is None and p.get_output_path() is None
    q = (p.video_path("in.mp4").output_path("out.avi").colorize(True).spatial_window_size(3)
         .sensitivity(2.5).filter_type(DiPsFilter.Sigmoid).chroma_filter(ChromaFilter.Red))
    assert q is p
    b = p.build()
    assert b is not p
    assert (b.get_video_path(), b.get_output_path(), b.colorize_, b.spatial_window_size_,
            b.sensitivity_, b.filter_type_, b.chroma_filter_) == (
        "in.mp4", "out.avi", True, 3, 2.5, DiPsFilter.Sigmoid, ChromaFilter.Red)


def test_series_conversions():
    a = np.array([[1, 2, 3, 1 << 32], [0, 0, 0, 3 << 31]], dtype=np.uint64)
    s = Series.from_array(a)
    assert np.array_equal(s.as_array(), a)
    assert list(s.si) == [1.0, 1.5]
    assert list(si_from_fixed([1 << 31])) == [0.5]
    assert s.sj_norm[0] == 2 / 510


def test_frame_geometry_checks():
    assert _frame_geometry(np.zeros((2, 3, 4, 3), np.uint8), PixelFormat.RGB8) == (2, 3, 4)
    assert _frame_geometry(np.zeros((2, 3, 4), np.uint8), PixelFormat.Gray8) == (2, 3, 4)
    assert _frame_geometry(np.zeros((2, 3, 4, 1), np.uint8), PixelFormat.Gray8) == (2, 3, 4)
    with pytest.raises(ValueError):
        _frame_geometry(np.zeros((2, 3, 4, 4), np.uint8), PixelFormat.RGB8)
    with pytest.raises(ValueError):
        _frame_geometry(np.zeros((3, 4, 3), np.uint8), PixelFormat.RGB8)


def test_modes_and_formats():
    assert int(Mode.Overall) == 0 and int(Mode.PerFrame) == 1
    assert [int(f) for f in PixelFormat] == [1, 3, 4]
