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


_COPY_CHECK = r"""
#include "copy_pool.h"
#include <cstdio>
#include <random>
int main() {
    std::mt19937_64 rng(7);
    std::vector<uint8_t> src(9u << 20), dst((9u << 20) + 64), want;
    for (auto& b : src) b = (uint8_t)rng();
    const size_t sizes[] = {0, 1, 31, 32, 127, 128, 129, 65535, 65536, 65537, 1u << 20, (4u << 20) + 77, 9u << 20};
    int bad = 0;
    for (int rep = 0; rep < 2; ++rep) {
        for (size_t n : sizes)
            for (size_t so = 0; so < 4; ++so)
                for (size_t dof = 0; dof < 40; dof += 13) {
                    if (so + n > src.size() || dof + n + 8 > dst.size()) continue;
                    std::fill(dst.begin(), dst.end(), 0xA5);
                    dips_host::host_copy(dst.data() + dof, src.data() + so, n);
                    for (size_t i = 0; i < dof; ++i) bad += dst[i] != 0xA5;
                    bad += std::memcmp(dst.data() + dof, src.data() + so, n) != 0;
                    for (size_t i = dof + n; i < dof + n + 8; ++i) bad += dst[i] != 0xA5;
                }
        std::fill(dst.begin(), dst.end(), 0);
        dips_host::pool_copy(dst.data() + 3, src.data() + 1, (9u << 20) - 1);
        bad += std::memcmp(dst.data() + 3, src.data() + 1, (9u << 20) - 1) != 0;
    }
    std::printf("bad=%d\n", bad);
    return bad != 0;
}
"""


def test_host_staging_copy_matches_memcpy(tmp_path):
    """copy_pool.h: the streaming staging copy (AVX2 non-temporal stores) and
    the pooled piecewise copy equal memcpy for every size class and source /
    destination alignment, and write nothing outside the destination range."""
    import os
    import shutil
    import subprocess
    if shutil.which("g++") is None:
        pytest.skip("no g++")
    csrc = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "dips_amd", "csrc")
    src = tmp_path / "copy_check.cpp"
    src.write_text(_COPY_CHECK)
    exe = tmp_path / "copy_check"
    subprocess.run(["g++", "-O2", "-std=c++17", "-pthread", f"-I{csrc}", str(src), "-o", str(exe)], check=True)
    r = subprocess.run([str(exe)], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0 and "bad=0" in r.stdout, r.stdout + r.stderr


_GEOM_CHECK = r"""
#include "host_stream.h"
#include <cstdio>
#include <cstdlib>
#include <string>
int main() {
    int bad = 0, cases = 0;
    const uint32_t heights[] = {1, 2, 3, 7, 29, 48, 480, 1080, 2160, 4320};
    const size_t rows[] = {4, 160, 164, 2560, 7680, 15360, 30720};
    // piece sizes: 4 MiB from 4 MiB frames up, quarters (>= 4 KiB, 64-B
    // multiples) below
    for (size_t fb : {(size_t)1, (size_t)4096, (size_t)12288, (size_t)1228800, (size_t)((4u << 20) - 1),
                      (size_t)(4u << 20), (size_t)33177600}) {
        const size_t pb = dips_host::piece_bytes(fb);
        ++cases;
        if (pb % 64 != 0 || pb < 4096 || pb > (4u << 20) || (fb >= (4u << 20) && pb != (4u << 20))) ++bad;
        if (fb >= 16384 && fb < (4u << 20) && (fb + pb - 1) / pb < 4) ++bad;
    }
    for (uint32_t hgt : heights) for (size_t row : rows) {
        dips_host::DirectGeom g;
        g.init(hgt, row);
        ++cases;
        if (g.k != dips_host::kDirectSplit) ++bad;
        // a frame of at least 16 KiB is cut into several stripes
        if ((size_t)hgt * row >= 16384 && hgt >= 8 && g.n_s < 2) ++bad;
        // stripes cover [0, height) in order, each non-empty
        uint32_t y = 0;
        for (uint32_t si = 0; si < g.n_s; ++si) {
            if (g.y0(si) != y || g.y1(si) <= g.y0(si)) { ++bad; break; }
            y = g.y1(si);
        }
        if (y != hgt) ++bad;
        // pieces cover each stripe's bytes exactly, cuts 64-B aligned inside the stripe
        for (uint32_t si = 0; si < g.n_s; ++si) {
            size_t at = (size_t)g.y0(si) * row;
            for (uint32_t j = 0; j < g.k; ++j) {
                size_t o, len;
                g.piece(si, j, o, len);
                if (o != at) { ++bad; break; }
                if (j + 1 < g.k && ((o + len - (size_t)g.y0(si) * row) % 64) != 0 && len) ++bad;
                at = o + len;
            }
            if (at != (size_t)g.y1(si) * row) ++bad;
        }
    }
    std::printf("cases=%d bad=%d\n", cases, bad);
    return bad != 0;
}
"""


def test_zero_copy_stripe_geometry(tmp_path):
    """host_stream.h piece_bytes and DirectGeom (the zero-copy per-frame
    pipeline): 4 MiB pieces from 4 MiB frames up, at least four pieces of a
    smaller frame; for every frame height and row size the stripes cover the
    frame's rows in order with none empty (several for any frame of 16 KiB or
    more), and each stripe's pieces cover its bytes exactly with cuts 64-B
    aligned inside the stripe."""
    import os
    import shutil
    import subprocess
    if shutil.which("g++") is None or not os.path.exists("/opt/rocm/include/hip/hip_runtime.h"):
        pytest.skip("no g++ or HIP headers")
    csrc = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "dips_amd", "csrc")
    src = tmp_path / "geom_check.cpp"
    src.write_text(_GEOM_CHECK)
    exe = tmp_path / "geom_check"
    subprocess.run(["g++", "-O1", "-std=c++17", "-pthread", "-D__HIP_PLATFORM_AMD__", "-I/opt/rocm/include",
                    f"-I{csrc}", str(src), "-o", str(exe), "-L/opt/rocm/lib", "-lamdhip64"], check=True)
    env = dict(os.environ, LD_LIBRARY_PATH="/opt/rocm/lib:" + os.environ.get("LD_LIBRARY_PATH", ""))
    r = subprocess.run([str(exe)], capture_output=True, text=True, timeout=120, env=env)
    assert r.returncode == 0 and "bad=0" in r.stdout, r.stdout + r.stderr


_KEYS_CHECK = r"""
#include "copy_pool.h"
#include <cstdio>
#include <random>
#include <vector>
int main() {
    std::mt19937_64 rng(11);
    int bad = 0;
    const size_t sizes[] = {0, 1, 7, 8, 9, 15, 16, 17, 33, 1000, 4099};
    for (int kb = 1; kb <= 2; ++kb)
        for (int nt = 0; nt < 2; ++nt)
            for (size_t npx : sizes)
                for (size_t dof = 0; dof < 40; dof += 4) {  // destination offsets in bytes (RGBA8: 4-aligned)
                    std::vector<uint8_t> keys(npx * kb + 1), dst(4 * npx + dof + 8, 0xA5);
                    for (auto& b : keys) b = (uint8_t)rng();
                    dips_host::expand_keys(dst.data() + dof, keys.data(), npx, kb, nt != 0);
                    for (size_t i = 0; i < dof; ++i) bad += dst[i] != 0xA5;
                    for (size_t p = 0; p < npx; ++p) {
                        const uint8_t r = keys[kb * p], g = kb == 1 ? r : keys[2 * p + 1];
                        const uint8_t want[4] = {r, g, r < g ? r : g, 255};
                        for (int c = 0; c < 4; ++c) bad += dst[dof + 4 * p + c] != want[c];
                    }
                    for (size_t i = dof + 4 * npx; i < dst.size(); ++i) bad += dst[i] != 0xA5;
                }
    std::printf("bad=%d\n", bad);
    return bad != 0;
}
"""


def test_expand_keys_rebuilds_rgba(tmp_path):
    """copy_pool.h expand_keys: the per-pixel keys of the zero-copy per-frame
    output (one byte gray / two bytes R, G; compat_main_host_kernel out_key)
    become (k, k, k, 255) / (r, g, min(r, g), 255) for every length and
    destination offset, AVX2 and streaming stores included, and nothing
    outside the destination is written."""
    import os
    import shutil
    import subprocess
    if shutil.which("g++") is None:
        pytest.skip("no g++")
    csrc = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "dips_amd", "csrc")
    src = tmp_path / "keys_check.cpp"
    src.write_text(_KEYS_CHECK)
    exe = tmp_path / "keys_check"
    subprocess.run(["g++", "-O2", "-std=c++17", "-pthread", f"-I{csrc}", str(src), "-o", str(exe)], check=True)
    r = subprocess.run([str(exe)], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0 and "bad=0" in r.stdout, r.stdout + r.stderr


_PACK_CHECK = r"""
#include "copy_pool.h"
#include <cstdio>
#include <random>
#include <vector>
int main() {
    std::mt19937_64 rng(5);
    int bad = 0;
    const size_t sizes[] = {0, 1, 7, 8, 15, 16, 17, 31, 33, 1000, 4099};
    for (int ib = 1; ib <= 2; ++ib)
        for (int ch = 0; ch < (ib == 1 ? 3 : 1); ++ch)
            for (int nt = 0; nt < 2; ++nt)
                for (size_t npx : sizes)
                    for (size_t so = 0; so < 12; so += 4) {
                        std::vector<uint8_t> src(4 * npx + so + 4), dst(ib * npx + 64, 0xA5);
                        for (auto& b : src) b = (uint8_t)rng();
                        dips_host::pack_frame(dst.data() + 32, src.data() + so, npx, ib, ch, nt != 0);
                        for (size_t i = 0; i < 32; ++i) bad += dst[i] != 0xA5;
                        for (size_t p = 0; p < npx; ++p) {
                            const uint8_t* px = src.data() + so + 4 * p;
                            const uint8_t mx = std::max(std::max(px[0], px[1]), px[2]);
                            const uint8_t mn = std::min(std::min(px[0], px[1]), px[2]);
                            if (ib == 2) bad += dst[32 + 2 * p] != mx || dst[32 + 2 * p + 1] != mn;
                            else bad += dst[32 + p] != px[ch];
                        }
                        for (size_t i = 32 + ib * npx; i < dst.size(); ++i) bad += dst[i] != 0xA5;
                    }
    std::printf("bad=%d\n", bad);
    return bad != 0;
}
"""


def test_pack_frame_for_the_zero_copy_input(tmp_path):
    """copy_pool.h pack_frame: the per-frame zero-copy input as the kernel
    reads it (compat_main_host_packed_kernel in_key) -- per-pixel (max, min)
    of R, G, B, or one chroma channel -- for every length, source offset and
    channel, AVX2 and streaming stores included, nothing written outside."""
    import os
    import shutil
    import subprocess
    if shutil.which("g++") is None:
        pytest.skip("no g++")
    csrc = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "dips_amd", "csrc")
    src = tmp_path / "pack_check.cpp"
    src.write_text(_PACK_CHECK)
    exe = tmp_path / "pack_check"
    subprocess.run(["g++", "-O2", "-std=c++17", "-pthread", f"-I{csrc}", str(src), "-o", str(exe)], check=True)
    r = subprocess.run([str(exe)], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0 and "bad=0" in r.stdout, r.stdout + r.stderr


def test_bench_kernel_name_matches_library_choice():
    """bench.py names the series_v2 instantiation the library runs, spelled
    as rocprofv3 prints it (ISI an int): run_series_device's choice of the
    intensity-sum form (series_abi.hip series_isi_form)."""
    import bench
    assert bench._v2_kernel_name(True, 8 / 255) == "series_v2_kernel<3, 0, 5, true, false, false, 1>"
    assert bench._v2_kernel_name(False, 8 / 255, with_map=True) == "series_v2_kernel<3, 0, 5, false, true, false, 1>"
    assert bench._v2_kernel_name(True, 0.0) == "series_v2_kernel<3, 0, 5, true, false, false, 0>"
    assert bench._series_isi(0.0) == 0 and bench._series_isi(0.03) == 0 and bench._series_isi(1 / 32) == 1
    assert bench._series_isi(1.0) == 1
